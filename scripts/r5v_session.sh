# two-rank rehearsal of the bench's N > 1 contract on one GPU (gloo collectives; the partitioned block needs RCCL and one GPU per rank)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo > gpurun_out/r5v_bench_2rank_gloo.json 2> gpurun_out/r5v_bench_2rank_gloo.err
