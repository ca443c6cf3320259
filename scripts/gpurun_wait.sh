#!/bin/bash
# Submit one gpurun call, re-submitting ONLY while the pool reports no free
# box / slot (exit status 3: nothing ran, nothing charged).  Any other status
# -- success, a failing command, a refusal -- ends it.  Usage:
#   scripts/gpurun_wait.sh TIMEOUT_S 'command' [max_tries]
t=$1; cmd=$2; tries=${3:-30}
for i in $(seq 1 "$tries"); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$cmd"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 90
done
exit 3
