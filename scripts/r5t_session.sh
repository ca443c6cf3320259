# direct-level threshold: 2 (default) vs 1 batch per top-down block
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=gpurun_out/r5t_direct_batches_ab.jsonl
for rep in 1 2; do
  for v in db2 db1; do
    for g in kron:22:16:1 kron:25:16:1 gnp:10000000::1; do
      LD_LIBRARY_PATH=build/var/$v timeout -k 10 240 python3 benchmarks/pair_latency.py --graph $g --pairs 64 --reps 5 --summary $v >> $O 2>>gpurun_out/r5t.err || exit 1
    done
  done
done
