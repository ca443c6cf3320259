#!/bin/bash
# One entry point for the GPU-box sessions (replaces the per-session
# r3*/r4*/r5*_session.sh scripts of rounds 3-4).  Run on the box through
# gpurun, e.g.
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
#            over 1k/10k/50k/100k x v1, v2 (np 4), v3 (--resident), v4 (np 4: ranks share the GPU over IPC)
#   prof     rocprofv3 --kernel-trace --stats of a short bench
#   pmc      one SQ counter pass (rocprofv3 --pmc) over the resident 100k workload (PMCGRAPH=spec: another graph)
#   benchab  driver-style headline bench (no extras) A/B over ABENV=<var> ABVALS="<v1> <v2>"
#            [ROUNDS=3 STEPS=20 WARMUP=5], one JSON line per run
#   stamp    cycle stamps of the 100k tiny resident server (BIBFS_TINY_STAMP: its stamped build)
#   distab   partitioned engine: local-group P = 1/2/4 per-round kernel vs exchange stamps
#            (SPECS / RANKS / PIPELINE / QUERIES / PROCS=1 / DEVSYNC override benchmarks/dist_rounds.py's defaults)
#   procs    partitioned engine as separate processes on the one GPU (IPC transport):
#            tests/test_gpu_dist_proc.py
#   pairab   A/B of one environment knob over pair latencies: ABENV=<var> ABVALS="<v1> <v2>"
#            GRAPHS="<spec> ..." [PAIRS=64 REPS=5 ROUNDS=2]; ABLIB="<dir1> <dir2>" instead
#            A/Bs library builds (LD_LIBRARY_PATH=build/var/<dir>, scripts/build_variants.sh)
#   trace    rocprofv3 --kernel-trace of pair_latency over GRAPHS (per-query kernel timelines)
#   kron     benchmarks/kron_scale.py over SCALES (default 20,22,24,26,27,28), resident server
#   stress   benchmarks/stress_resident.py
#   dstress  benchmarks/stress_dist_local.py --procs (partitioned engine as processes, answers vs the CPU)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG="${TAG:-r6}"
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
      TIERS="v1 v2 v3 v4" REPEAT=20 WARMUP=5 NP=4 V4NP=4 PER_RUN_TIMEOUT=120 \
        LOGDIR=$O/${TAG}_suite_logs CSV=$O/${TAG}_benchmark_results.csv \
        $T 900 bash scripts/benchmark_test.sh $O/${TAG}_graphs > $O/${TAG}_benchmark_table.txt 2>&1 ;;
    prof)
      $T 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_prof -o prof -- \
        python3 bench.py --steps 20 --warmup 5 --extra-steps 50 --batch 0 --no-cpu-ref \
        > $O/${TAG}_prof_bench.json 2> $O/${TAG}_prof_bench.err ;;
    benchab)  # headline bench (no extras), interleaved over ABENV=ABVALS, ROUNDS times
      for r in $(seq 1 ${ROUNDS:-3}); do for v in $ABVALS; do
        env $ABENV=$v $T 300 python3 bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARMUP:-5} \
          --extra-graph '' --dist-graphs '' --batch 0 --no-cpu-ref 2>> $O/${TAG}_benchab.err |
          python3 -c "import json,sys; d=json.loads(sys.stdin.read()); x=d['detail']; print(json.dumps({'$ABENV': '$v', 'round': $r, 'query_ms': x['query_ms'], 'device_ms': x['device_ms_per_query'], 'value': d['value'], 'tiny_overflows': x['tiny_overflows']}))" \
          >> $O/${TAG}_benchab.jsonl || exit 1
      done; done ;;
    stamp)
      BIBFS_TINY_STAMP=1 $T 120 ./build/bin/bibfs_hip gnp:100000::6 0 99999 --verify --resident --repeat 8 \
        > $O/${TAG}_stamp_100k.txt 2>&1 ;;
    pmc)  # PMCCTRS: another counter set (<= 8 SQ); PMCLIB: a build/var/<dir> library build
      local ctrs=${PMCCTRS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES"}
      env ${PMCLIB:+LD_LIBRARY_PATH=build/var/$PMCLIB} timeout -s KILL 120 rocprofv3 --output-format csv --pmc $ctrs \
        -d $O/${TAG}_pmc_sq -- \
        python3 benchmarks/pmc_100k.py --mode resident ${PMCGRAPH:+--graph $PMCGRAPH} > $O/${TAG}_pmc_sq.log 2>&1 ;;
    dstress)
      $T 900 python3 -u benchmarks/stress_dist_local.py --procs ${RANKS:+--ranks $RANKS} ${QUERIES:+--queries $QUERIES} \
        > $O/${TAG}_dstress.jsonl 2> $O/${TAG}_dstress.err ;;
    distab)
      $T 900 python3 benchmarks/dist_rounds.py ${SPECS:+--specs $SPECS} ${RANKS:+--ranks $RANKS} \
        ${PIPELINE:+--pipeline $PIPELINE} ${QUERIES:+--queries $QUERIES} ${PROCS:+--procs} ${DEVSYNC:+--dev-sync $DEVSYNC} \
        > $O/${TAG}_dist_rounds.jsonl 2> $O/${TAG}_dist_rounds.err ;;
    procs)
      $T 900 $PT -m gpu tests/test_gpu_dist_proc.py > $O/${TAG}_procs.log 2>&1 ;;
    pairab)
      local out=$O/${TAG}_pairab.jsonl
      for rep in $(seq 1 "${ROUNDS:-2}"); do
        for v in ${ABVALS:-$ABLIB}; do
          for g in $GRAPHS; do
            if [ -n "$ABLIB" ]; then
              LD_LIBRARY_PATH=build/var/$v $T 240 python3 benchmarks/pair_latency.py --graph "$g" \
                --pairs "${PAIRS:-64}" --reps "${REPS:-5}" --summary "$v" >> $out 2>> $O/${TAG}_pairab.err || return 1
            else
              env "$ABENV=$v" $T 240 python3 benchmarks/pair_latency.py --graph "$g" \
                --pairs "${PAIRS:-64}" --reps "${REPS:-5}" --summary "$ABENV=$v" >> $out 2>> $O/${TAG}_pairab.err || return 1
            fi
          done
        done
      done ;;
    trace)
      for g in ${GRAPHS:-gnp:10000000::1 kron:22:16:1}; do
        local t; t=$(echo "$g" | tr ':' '_')
        $T 300 rocprofv3 --kernel-trace --output-format csv -d $O/${TAG}_tr_$t -o run -- \
          python3 benchmarks/pair_latency.py --graph "$g" --pairs 32 --reps 3 --summary trace \
          > $O/${TAG}_tr_$t.jsonl 2> $O/${TAG}_tr_$t.err || return 1
      done ;;
    kron)
      $T 900 python3 benchmarks/kron_scale.py --scales "${SCALES:-20,22,24,26,27,28}" --queries 48 --resident \
        > $O/${TAG}_kron_scale.jsonl 2> $O/${TAG}_kron_scale.err ;;
    stress)
      $T 900 python3 -u benchmarks/stress_resident.py > $O/${TAG}_stress.jsonl 2> $O/${TAG}_stress.err ;;
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
