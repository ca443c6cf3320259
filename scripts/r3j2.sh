#!/bin/bash
# Round 3j2: tiny server lockstep cap re-tuned with the x4 + speculative loads:
# 768 / 1024 (default) / 1536 frontier edges; tiny GPU tests on each variant,
# then an interleaved latency A/B, 1920 queries each, twice.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="timeout -k 10"
for v in lock768 lock1536; do
  LD_LIBRARY_PATH=build/var/$v $T 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py -k "tiny or resident" > gpurun_out/rj_tests_$v.log 2>&1
  rc=$?; echo "tests $v rc=$rc"; [ $rc -le 1 ] || exit $rc
done
out=gpurun_out/rj_tiny_lock_ab.jsonl
: > $out
for rep in 1 2; do
  for v in base lock768 lock1536; do
    LD_LIBRARY_PATH=build/var/$v $T 90 python3 benchmarks/tiny_latency.py --reps 30 > gpurun_out/rj_one.jsonl 2> gpurun_out/rj_one_$v.err || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/rj_one.jsonl').readline()); d['variant']='$v'; print(json.dumps(d))" >> $out
  done
done
echo done
