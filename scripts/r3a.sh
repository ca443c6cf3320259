set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py -k "tiny or resident" > gpurun_out/r3a_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r3a_tests.log; exit 1; }
tail -3 gpurun_out/r3a_tests.log
timeout -k 10 200 python -u benchmarks/tiny_latency.py --reps 50 > gpurun_out/r3a_lat.jsonl 2> gpurun_out/r3a_lat.err || { echo LAT_FAILED; tail -20 gpurun_out/r3a_lat.err; exit 1; }
cat gpurun_out/r3a_lat.jsonl
BIBFS_NO_TINY=1 timeout -k 10 200 python -u benchmarks/tiny_latency.py --reps 50 > gpurun_out/r3a_lat_lds.jsonl 2>&1 || { echo LAT2_FAILED; exit 1; }
cat gpurun_out/r3a_lat_lds.jsonl
BIBFS_TINY_STAMP=1 timeout -k 10 120 ./build/bin/bibfs_hip gnp:100000::6 0 99999 --resident --repeat 10 > gpurun_out/r3a_stamp.txt 2>&1 || { echo STAMP_FAILED; tail gpurun_out/r3a_stamp.txt; exit 1; }
tail -15 gpurun_out/r3a_stamp.txt
