# grid top-down: packed adjacency on small levels + no trailing ticket (build/var gp1 = default, gp0 = column loads) + engine GPU tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py > gpurun_out/r5g_pytest.log 2>&1 || exit 1
O=gpurun_out/r5g_gridpadj_ab.jsonl
for rep in 1 2; do
  for v in gp1 gp0; do
    for g in gnp:10000000::1 gnp:3000000::4 kron:22:16:1; do
      LD_LIBRARY_PATH=build/var/$v timeout -k 10 240 python3 benchmarks/pair_latency.py --graph $g --pairs 64 --reps 5 --summary $v >> $O 2>>gpurun_out/r5g.err || exit 1
    done
  done
done
