# partitioned-engine stress on the local group: P = 2, 3, 4, 8 ranks on one GPU, hops vs the CPU engine, paths validated collectively
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python3 -u benchmarks/stress_dist_local.py --queries 512 > gpurun_out/r5p_stress_dist.jsonl 2> gpurun_out/r5p_stress_dist.err || exit 1
timeout -k 10 900 python3 -u benchmarks/stress_dist_local.py --queries 512 --overlap 1 > gpurun_out/r5p_stress_dist_overlap.jsonl 2> gpurun_out/r5p_stress_dist_overlap.err
