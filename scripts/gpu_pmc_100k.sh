#!/bin/bash
# Counter passes (one rocprofv3 --pmc run each, within the per-block limits)
# over the clean 100k headline workload (benchmarks/pmc_100k.py), one-shot and
# resident; summarised by tools/py/pmc_summary.py.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
W="python3 benchmarks/pmc_100k.py"
P="timeout -s KILL 120 rocprofv3 --output-format csv"
for mode in oneshot resident; do
  $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES \
     -d gpurun_out/pmc100k_${mode}_sq -- $W --mode $mode > gpurun_out/pmc100k_${mode}_sq.log 2>&1 && \
  $P --pmc TCC_HIT_sum TCC_MISS_sum TCC_READ_sum TCC_WRITE_sum \
     -d gpurun_out/pmc100k_${mode}_tcc -- $W --mode $mode > gpurun_out/pmc100k_${mode}_tcc.log 2>&1 && \
  $P --pmc TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum \
     -d gpurun_out/pmc100k_${mode}_ea -- $W --mode $mode > gpurun_out/pmc100k_${mode}_ea.log 2>&1 || exit 1
done
