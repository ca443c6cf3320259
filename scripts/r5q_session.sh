# LDS engine phase stamps on 10M G(n, p) (one-shot k_lds_bibfs stamped build, BIBFS_STAMP)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for p in "0 9999999" "123456 7654321" "2000000 8000000"; do
  BIBFS_STAMP=1 timeout -k 10 120 ./build/bin/bibfs_hip gnp:10000000::1 $p --trace --repeat 3 --verify >> gpurun_out/r5q_stamp_10m.txt 2>&1 || exit 1
done
