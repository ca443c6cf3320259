# grid publish walk time on hand-off searches (HostResult::rt_walk)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for g in gnp:10000000::1 kron:22:16:1 gnp:3000000::4; do
  timeout -k 10 240 python3 benchmarks/pair_latency.py --graph $g --pairs 64 --reps 5 --summary walk >> gpurun_out/r5h_walk.jsonl 2>>gpurun_out/r5h.err || exit 1
done
