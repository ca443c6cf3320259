# direct hub levels (BIBFS_GRID_HUB_DIRECT 0 / 1 / 2) A/B on Kronecker 22 and 25
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=gpurun_out/r4t_hubdirect_ab.jsonl
for d in 1 0 2 1 0 2; do
  BIBFS_GRID_HUB_DIRECT=$d timeout -k 10 240 python3 benchmarks/pair_latency.py --graph kron:22:16:1 --pairs 64 --reps 5 --summary direct$d >> $O 2>>gpurun_out/r4t.err || exit 1
done
for d in 1 0; do
  BIBFS_GRID_HUB_DIRECT=$d timeout -k 10 240 python3 benchmarks/pair_latency.py --graph kron:25:16:1 --pairs 32 --reps 5 --summary k25direct$d >> $O 2>>gpurun_out/r4t.err || exit 1
done
