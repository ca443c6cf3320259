# final kernel traces of resident hand-off searches: 10M G(n, p) and Kronecker 22
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for g in gnp:10000000::1 kron:22:16:1; do
  t=$(echo $g | tr ':' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5s_tr_$t -o run -- \
    python3 benchmarks/pair_latency.py --graph $g --pairs 32 --reps 3 --summary trace > gpurun_out/r5s_$t.jsonl 2> gpurun_out/r5s_$t.err || exit 1
done
