# kernel trace of resident 10M / Kronecker 22 searches (grid level timeline)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for g in gnp:10000000::1 kron:22:16:1; do
  t=$(echo $g | tr ':' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4r_tr_$t -o run -- \
    python3 benchmarks/pair_latency.py --graph $g --pairs 32 --reps 3 --summary trace > gpurun_out/r4r_$t.jsonl 2> gpurun_out/r4r_$t.err || exit 1
done
