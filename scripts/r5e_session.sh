# dist engine: one-chunk frontiers spread over every expand block -- GPU dist tests + local-group round stamps
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dist_local.py tests/test_gpu_dist_and_tools.py > gpurun_out/r5e_pytest.log 2>&1 || exit 1
timeout -k 10 400 python3 benchmarks/dist_rounds.py --specs kron:22,gnp:1000000::2 --ranks 2,4 --overlap 0 --queries 16 > gpurun_out/r5e_dist_rounds.jsonl 2> gpurun_out/r5e_dist_rounds.err
