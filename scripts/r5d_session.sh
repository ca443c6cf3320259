# direct edge-parallel levels widened to small heavy frontiers without hubs: A/B (BIBFS_GRID_HUB_DIRECT 1 / 0) + engine GPU tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py > gpurun_out/r5d_pytest.log 2>&1 || exit 1
O=gpurun_out/r5d_direct2_ab.jsonl
for rep in 1 2; do
  for d in 1 0; do
    for g in kron:22:16:1 kron:25:16:1 gnp:10000000::1; do
      BIBFS_GRID_HUB_DIRECT=$d timeout -k 10 240 python3 benchmarks/pair_latency.py --graph $g --pairs 48 --reps 5 --summary direct$d >> $O 2>>gpurun_out/r5d.err || exit 1
    done
  done
done
