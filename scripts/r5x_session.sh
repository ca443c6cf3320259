# final-tree local-group round stamps, overlap off and on
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python3 benchmarks/dist_rounds.py --specs gnp:1000000::2,kron:22 --ranks 2,4 --overlap 0,1 --queries 16 > gpurun_out/r5x_dist_rounds.jsonl 2> gpurun_out/r5x_dist_rounds.err
