#!/bin/bash
# Round 3i2: tiny server, speculative next-record loads in all-wave rounds
# (BIBFS_TINY_SPEC_ALL=1) re-measured now that the first-edge loads are two
# 16-byte loads (x4 default): GPU tiny/resident tests on the variant, then an
# interleaved latency A/B, 1920 queries each, twice.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="timeout -k 10"
LD_LIBRARY_PATH=build/var/specall $T 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py -k "tiny or resident" > gpurun_out/ri_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ] || exit $rc
out=gpurun_out/ri_tiny_specall_ab.jsonl
: > $out
for rep in 1 2; do
  for v in base specall; do
    LD_LIBRARY_PATH=build/var/$v $T 90 python3 benchmarks/tiny_latency.py --reps 30 > gpurun_out/ri_one.jsonl 2> gpurun_out/ri_one_$v.err || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/ri_one.jsonl').readline()); d['variant']='$v'; print(json.dumps(d))" >> $out
  done
done
echo done
