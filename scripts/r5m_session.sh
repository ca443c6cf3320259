# 8-byte packed adjacency (BIBFS_PADJ8 1 / 0) + engine GPU tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py > gpurun_out/r5m_pytest.log 2>&1 || exit 1
O=gpurun_out/r5m_padj8_ab.jsonl
for rep in 1 2; do
  for p8 in 1 0; do
    for g in gnp:10000000::1 gnp:3000000::4 gnp:1000000::2; do
      BIBFS_PADJ8=$p8 timeout -k 10 240 python3 benchmarks/pair_latency.py --graph $g --pairs 64 --reps 5 --summary padj8_$p8 >> $O 2>>gpurun_out/r5m.err || exit 1
    done
  done
done
