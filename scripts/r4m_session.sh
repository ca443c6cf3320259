# pair-latency splits (LDS phase vs grid levels) of the bench extras, then the
# single-wave 4-item A/B of the tiny server (build/var/sw2, sw4)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=gpurun_out/${TAG:-r4n}_split.jsonl
for g in gnp:10000000::1 kron:22:16:1; do
  timeout -k 10 240 python3 benchmarks/pair_latency.py --graph $g --pairs 64 --reps 5 --summary split >> $O 2>>gpurun_out/${TAG:-r4n}.err || exit 1
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py -k "tiny or resident" > gpurun_out/${TAG:-r4n}_pytest.log 2>&1 || exit 1
for d in build/var/sw4; do
  LD_LIBRARY_PATH=$d timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py -k "tiny" > gpurun_out/${TAG:-r4n}_pytest_sw4.log 2>&1 || exit 1
done
bash scripts/ab_tiny.sh > gpurun_out/${TAG:-r4n}_ab_tiny.log 2>&1 && cp gpurun_out/ab_tiny.jsonl gpurun_out/${TAG:-r4n}_ab_tiny.jsonl
