# resident-server stress on the final tree: 4000 back-to-back queries per graph, hops vs the CPU engine
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python3 -u benchmarks/stress_resident.py > gpurun_out/r5l_stress.jsonl 2> gpurun_out/r5l_stress.err
