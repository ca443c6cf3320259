#!/bin/bash
# One entry point for the GPU-box sessions (replaces the per-session r3*.sh
# scripts of round 3).  Run on the box through gpurun, e.g.
#
#   gpurun --timeout 900 -- 'bash scripts/gpu_tasks.sh pytest smoke bench'
#
# Each task writes under gpurun_out/<TAG>_* (TAG defaults to "r4"), runs every
# GPU step under its own `timeout -k 10`, and the chain stops at the first
# failing task (no retries after a fault, abort or time limit).
#
# tasks:
#   pytest   whole GPU test suite (one process)
#   smoke    __graft_entry__.smoke()
#   bench    driver-style bench: python bench.py --gpus 1 --steps 20 --warmup 5
#   suite    reference suite table (C21): scripts/make_graphs + scripts/benchmark_test.sh
#            over 1k/10k/50k/100k x v1, v2 (np 4), v3 (--resident), v4 (np 1)
#   prof     rocprofv3 --kernel-trace --stats of a short bench
#   pmc      one SQ counter pass (rocprofv3 --pmc) over the resident 100k workload
#   stamp    cycle stamps of the 100k tiny resident server (BIBFS_TINY_STAMP: its stamped build)
#   distab   partitioned engine: local-group P = 1/2/4 per-round kernel vs exchange stamps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG="${TAG:-r4}"
T="timeout -k 10"
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
O=gpurun_out

run_task() {
  case "$1" in
    pytest)
      $T 900 $PT -m gpu tests > $O/${TAG}_pytest.log 2>&1 ;;
    smoke)
      $T 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 ;;
    bench)
      $T 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err ;;
    suite)
      SIZES="1000 10000 50000 100000" SEED=1 bash scripts/make_graphs $O/${TAG}_graphs > $O/${TAG}_make_graphs.log 2>&1 &&
      TIERS="v1 v2 v3 v4" REPEAT=20 WARMUP=5 NP=4 NGPU=1 PER_RUN_TIMEOUT=120 \
        LOGDIR=$O/${TAG}_suite_logs CSV=$O/${TAG}_benchmark_results.csv \
        $T 900 bash scripts/benchmark_test.sh $O/${TAG}_graphs > $O/${TAG}_benchmark_table.txt 2>&1 ;;
    prof)
      $T 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_prof -o prof -- \
        python3 bench.py --steps 20 --warmup 5 --extra-steps 50 --batch 0 --no-cpu-ref \
        > $O/${TAG}_prof_bench.json 2> $O/${TAG}_prof_bench.err ;;
    stamp)
      BIBFS_TINY_STAMP=1 $T 120 ./build/bin/bibfs_hip gnp:100000::6 0 99999 --verify --resident --repeat 8 \
        > $O/${TAG}_stamp_100k.txt 2>&1 ;;
    pmc)
      timeout -s KILL 120 rocprofv3 --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
        SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES -d $O/${TAG}_pmc_sq -- \
        python3 benchmarks/pmc_100k.py --mode resident > $O/${TAG}_pmc_sq.log 2>&1 ;;
    distab)
      $T 600 python3 benchmarks/dist_rounds.py > $O/${TAG}_dist_rounds.jsonl 2> $O/${TAG}_dist_rounds.err ;;
    *)
      echo "unknown task $1" >&2; return 2 ;;
  esac
}

for t in "$@"; do
  echo "== $t $(date +%T)"
  run_task "$t"
  rc=$?
  echo "== $t rc=$rc $(date +%T)"
  [ $rc -eq 0 ] || exit $rc
done
