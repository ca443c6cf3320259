# bucketed LDS hash probing (BIBFS_KNOB_HASH_BUCKET; build/var hb1 = default, hb0 = one CAS per slot) + engine GPU tests + stress
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py > gpurun_out/r5r_pytest.log 2>&1 || exit 1
timeout -k 10 600 python3 -u benchmarks/stress_resident.py --graphs gnp:3000000::4,gnp:10000000::1,kron:20:16:2 --queries 2000 > gpurun_out/r5r_stress.jsonl 2> gpurun_out/r5r_stress.err || exit 1
O=gpurun_out/r5r_hashbucket_ab.jsonl
for rep in 1 2; do
  for v in hb1 hb0; do
    for g in gnp:10000000::1 gnp:3000000::4 gnp:1000000::2 kron:22:16:1; do
      LD_LIBRARY_PATH=build/var/$v timeout -k 10 240 python3 benchmarks/pair_latency.py --graph $g --pairs 64 --reps 5 --summary $v >> $O 2>>gpurun_out/r5r.err || exit 1
    done
  done
done
