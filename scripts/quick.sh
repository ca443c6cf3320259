set -o pipefail
B=./build/bin/bibfs_hip
timeout -k 10 300 ./build/bin/bibfs_selftest gnp:1000::1 gnp:100000::6 gnp:1000000::2 rmat:65536:1048576:3 kron:16:16:2 > gpurun_out/selftest.log 2>&1 && \
BIBFS_STAMP=1 timeout -k 10 60 $B gnp:100000::6 0 99999 --trace --repeat 5 --verify > gpurun_out/stamp.log 2>&1 && \
: > gpurun_out/lat.txt && \
for g in "gnp:100000::6 0 99999" "gnp:1000000::2 0 999999" "gnp:10000000::1 0 9999999"; do
  timeout -k 10 120 $B $g --json --repeat 200 >> gpurun_out/lat.txt 2>&1 && \
  timeout -k 10 120 $B $g --json --repeat 200 --resident >> gpurun_out/lat.txt 2>&1 || exit 1
done
