set -o pipefail
B=./build/bin/bibfs_hip
timeout -k 5 30 $B gnp:100000::6 0 99999 --repeat 5 > gpurun_out/oneshot.txt 2>&1 && \
BIBFS_DEBUG=1 timeout -k 5 20 $B gnp:100000::6 0 99999 --repeat 5 --resident > gpurun_out/res1.txt 2> gpurun_out/res1.err
