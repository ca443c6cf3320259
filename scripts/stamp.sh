set -o pipefail
B=./build/bin/bibfs_hip
timeout -k 10 240 ./build/bin/bibfs_selftest gnp:1000::1 gnp:100000::6 gnp:131072::3 gnp:1000000::2 rmat:65536:1048576:3 kron:16:16:2 > gpurun_out/selftest.log 2>&1 && \
BIBFS_STAMP=1 timeout -k 10 60 $B gnp:100000::6 0 99999 --verify --trace --repeat 5 > gpurun_out/stamp.log 2>&1 && \
timeout -k 10 60 $B gnp:100000::6 0 99999 --json --repeat 200 > gpurun_out/lat.txt 2>&1 && \
timeout -k 10 60 $B gnp:100000::6 0 99999 --json --repeat 200 --no-lockstep >> gpurun_out/lat.txt 2>&1 && \
timeout -k 10 60 $B gnp:1000000::2 0 999999 --json --repeat 100 >> gpurun_out/lat.txt 2>&1
