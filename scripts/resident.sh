set -o pipefail
B=./build/bin/bibfs_hip
timeout -k 10 300 ./build/bin/bibfs_selftest gnp:1000::1 gnp:100000::6 gnp:1000000::2 rmat:65536:1048576:3 kron:16:16:2 > gpurun_out/selftest.log 2>&1 && \
bash scripts/ab_env.sh "oneshot=X=1" > /dev/null && mv gpurun_out/ab_env.txt gpurun_out/ab_oneshot.txt && \
for g in "gnp:100000::6 0 99999" "gnp:1000000::2 0 999999" "gnp:10000000::1 0 9999999"; do
  timeout -k 10 90 $B $g --json --repeat 300 --resident >> gpurun_out/resident.txt 2>&1 || exit 1
done
