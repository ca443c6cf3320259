# auto chain on a hub graph: one search at a time, debug prints (BIBFS_DEBUG)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for lv in 1 2 3 8; do
  BIBFS_DEBUG=1 timeout -k 10 70 python3 benchmarks/auto_chain_repro.py --levels $lv --pairs 32 > gpurun_out/r4q_lv$lv.log 2>&1
  rc=$?; echo "lv$lv rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
