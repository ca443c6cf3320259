#!/bin/bash
# Kronecker sweep on one GPU + rocprofv3 counter passes (each its own run,
# --pmc only with --kernel-trace-free output; counters per block within limits).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="timeout -k 10"
$T 600 python -u benchmarks/kron_scale.py --scales 20,22,24,26,27 > gpurun_out/kron.jsonl 2> gpurun_out/kron.err && \
{ $T 60 rocprofv3 --list-avail > gpurun_out/pmc_avail.txt 2>&1 || true; } && \
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc_sq -- python3 benchmarks/pmc_workload.py > gpurun_out/pmc_sq.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_tcc -- python3 benchmarks/pmc_workload.py > gpurun_out/pmc_tcc.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -- python3 benchmarks/pmc_workload.py > gpurun_out/pmc_fetch.log 2>&1 && \
$T 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
