#!/bin/bash
# Run one command on the GPU box via gpurun and print its verdict.
# usage: scripts/gpu.sh TIMEOUT_S 'command'
t=$1; shift
/usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > /tmp/gpurun_last.txt 2>&1
rc=$?
tail -3 /tmp/gpurun_last.txt
python3 - <<'PY'
import json
d = json.load(open("/root/repo/gpurun_out/.last_call.json"))
print("verdict:", d.get("status"), "rc", d.get("rc"), d.get("msg", "")[:200], "run_s", d.get("run_s"))
PY
exit $rc
