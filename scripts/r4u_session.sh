# auto chain with direct hub levels on hub graphs: GPU tests + Kronecker 22 / 25 host vs auto A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py -k "auto or resident or handoff or grid" > gpurun_out/r4v_pytest.log 2>&1 || exit 1
O=gpurun_out/r4v_auto_hub_ab.jsonl
for md in 64 1000000000 64 1000000000; do
  BIBFS_AUTO_MAX_DEG=$md timeout -k 10 240 python3 benchmarks/pair_latency.py --graph kron:22:16:1 --pairs 64 --reps 5 --summary automaxdeg$md >> $O 2>>gpurun_out/r4v.err || exit 1
done
for md in 64 1000000000; do
  BIBFS_AUTO_MAX_DEG=$md timeout -k 10 240 python3 benchmarks/pair_latency.py --graph kron:25:16:1 --pairs 32 --reps 5 --summary k25automaxdeg$md >> $O 2>>gpurun_out/r4v.err || exit 1
done
