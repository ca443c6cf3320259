#!/bin/bash
# Round 3, final HEAD: tiny-server phase stamps and counter passes on the 100k
# headline (resident server), one rocprofv3 --pmc run per pass.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
BIBFS_TINY_STAMP=1 timeout -k 10 120 ./build/bin/bibfs_hip gnp:100000::6 0 99999 --resident --repeat 8 > gpurun_out/rp_stamp.txt 2>&1 || exit $?
W="python3 benchmarks/pmc_100k.py"
P="timeout -s KILL 120 rocprofv3 --output-format csv"
$P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES \
   -d gpurun_out/rp_sq -- $W --mode resident > gpurun_out/rp_sq.log 2>&1 || exit $?
$P --pmc TCC_HIT_sum TCC_MISS_sum TCC_READ_sum TCC_WRITE_sum -d gpurun_out/rp_tcc -- $W --mode resident > gpurun_out/rp_tcc.log 2>&1 || exit $?
echo done
