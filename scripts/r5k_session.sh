# evidence runs on the final round-4 tree: Kronecker scale sweep through the resident server,
# the reference suite table, and SQ counters of the 10M LDS-server workload
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python3 benchmarks/kron_scale.py --scales 20,22,24,26,27,28 --queries 48 --resident > gpurun_out/r5k_kron_scale.jsonl 2> gpurun_out/r5k_kron_scale.err || exit 1
TAG=r5k bash scripts/gpu_tasks.sh suite || exit 1
timeout -s KILL 180 rocprofv3 --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
  SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES -d gpurun_out/r5k_pmc10m -- \
  python3 benchmarks/pmc_100k.py --mode resident --graph gnp:10000000::1 --queries 256 > gpurun_out/r5k_pmc10m.log 2>&1
