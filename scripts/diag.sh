set -o pipefail
B=./build/bin/bibfs_hip
T="timeout -k 10 60"
$T $B gnp:100000::6 0 99999 --trace --no-lockstep --repeat 1 --verify > gpurun_out/diag_nolock.log 2>&1 && \
$T $B gnp:100000::6 0 99999 --trace --repeat 1 --verify > gpurun_out/diag_lock.log 2>&1 && \
$T $B gnp:100000::6 0 99999 --trace --side alternate --no-lockstep --repeat 1 --verify > gpurun_out/diag_alt.log 2>&1
