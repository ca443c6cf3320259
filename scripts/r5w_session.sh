# SQ counters of the Kronecker 22 resident workload (direct edge-parallel hub levels)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -s KILL 180 rocprofv3 --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
  SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES -d gpurun_out/r5w_pmckron -- \
  python3 benchmarks/pmc_100k.py --mode resident --graph kron:22:16:1 --queries 256 > gpurun_out/r5w_pmckron.log 2>&1
