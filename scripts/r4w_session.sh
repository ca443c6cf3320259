# LDS engine: all-wave rounds on hash sets with the global queue (default now) vs off (build/var/whg0)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py tests/test_gpu_dist_and_tools.py > gpurun_out/r4y_pytest.log 2>&1 || exit 1
O=gpurun_out/r4y_whg_ab.jsonl
for rep in 1 2; do
  for v in whg1 whg0; do
    for g in gnp:10000000::1 gnp:1000000::2 kron:22:16:1 gnp:3000000::4; do
      LD_LIBRARY_PATH=build/var/$v timeout -k 10 240 python3 benchmarks/pair_latency.py --graph $g --pairs 64 --reps 5 --summary $v >> $O 2>>gpurun_out/r4y.err || exit 1
    done
  done
done
