#!/bin/bash
# A/B of partitioned-engine variants in build/var_dist/NAME/libbibfs.so
# (world size 1 over RCCL, benchmarks/dist_ab.py, spec_rounds 1), interleaved.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_dist.txt
: > $out
for rep in 1 2; do
  for d in build/var_dist/*/; do
    v=$(basename $d)
    LD_LIBRARY_PATH=$d timeout -k 10 240 python3 benchmarks/dist_ab.py --specs "${SPECS:-gnp:1000000::2,kron:22,kron:25}" \
        --modes 1 --queries 32 --reps 2 2>/dev/null | grep '^{' | python3 -c '
import json, sys
for l in sys.stdin:
    d = json.loads(l)
    print(sys.argv[1], d["spec"], "median %.4f mean %.4f device %.4f" % (d["median_query_ms"], d["mean_query_ms"], d["median_device_ms"]))' $v >> $out || exit 1
  done
done
