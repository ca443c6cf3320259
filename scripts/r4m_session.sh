# GPU tests of the single-GPU engine, pair-latency splits (LDS phase vs grid
# levels) of the bench extras with 1 / 2 / 3 device-planned grid levels
# (BIBFS_AUTO_LEVELS), then the single-wave 4-item A/B of the tiny server
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
G=${TAG:-r4o}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py tests/test_gpu_dist_and_tools.py > gpurun_out/${G}_pytest.log 2>&1 || exit 1
O=gpurun_out/${G}_split.jsonl
for lv in 1 2 3 2 1; do
  BIBFS_AUTO_LEVELS=$lv timeout -k 10 240 python3 benchmarks/pair_latency.py --graph gnp:10000000::1 --pairs 64 --reps 5 --summary levels$lv >> $O 2>>gpurun_out/${G}.err || exit 1
done
for md in 64 1000000000 64 1000000000; do
  BIBFS_AUTO_MAX_DEG=$md timeout -k 10 240 python3 benchmarks/pair_latency.py --graph kron:22:16:1 --pairs 64 --reps 5 --summary automaxdeg$md >> $O 2>>gpurun_out/${G}.err || exit 1
done
for d in build/var/sw4; do
  LD_LIBRARY_PATH=$d timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py -k "tiny" > gpurun_out/${G}_pytest_sw4.log 2>&1 || exit 1
done
bash scripts/ab_tiny.sh > gpurun_out/${G}_ab_tiny.log 2>&1 && cp gpurun_out/ab_tiny.jsonl gpurun_out/${G}_ab_tiny.jsonl
