# round 3: tiny server stamps + tests + latency + driver-style bench + direction A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
BIBFS_TINY_STAMP=1 timeout -k 10 120 ./build/bin/bibfs_hip gnp:100000::6 0 99999 --resident --repeat 6 > $O/r3c_stamp.txt 2>&1 || { echo STAMP_FAILED; tail $O/r3c_stamp.txt; exit 1; }
tail -4 $O/r3c_stamp.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py -k "tiny or resident or unbalanced or streamed or lds_and_grid" > $O/r3c_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/r3c_tests.log; exit 1; }
tail -2 $O/r3c_tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dist_local.py -k "shards or out_of_range" > $O/r3c_dist.log 2>&1 || { echo DIST_FAILED; tail -30 $O/r3c_dist.log; exit 1; }
tail -2 $O/r3c_dist.log
timeout -k 10 200 python -u benchmarks/tiny_latency.py --reps 50 > $O/r3c_lat.jsonl 2> $O/r3c_lat.err || { echo LAT_FAILED; tail -20 $O/r3c_lat.err; exit 1; }
cat $O/r3c_lat.jsonl
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/r3c_bench.json 2> $O/r3c_bench.err || { echo BENCH_FAILED; tail -20 $O/r3c_bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/r3c_bench.json').read().strip().splitlines()[-1]);x=d['detail'];print('value',d['value'],'ms',d['ms_per_step'],'dev',x['device_ms_per_query'],'cpu',x['cpu_serial_query_ms'],x['cpu_serial_ms'],'launch',x['server_launch_ms']);[print(k,v.get('ms_per_query'),v.get('single_gpu_ms'),v.get('speedup_vs_single_gpu')) for k,v in x['partitioned'].items()];[print(k,v.get('ms_per_step')) for k,v in x['extra'].items()]"
for dir in auto topdown bottomup; do
  timeout -k 10 200 python -u benchmarks/kron_scale.py --scales 20,22,24 --queries 16 --direction $dir >> $O/r3c_dir_ab.jsonl 2>>$O/r3c_dir_ab.err || { echo DIR_FAILED; exit 1; }
done
timeout -k 10 200 python -u benchmarks/kron_scale.py --scales 20,22,24 --queries 16 --alpha 4 --beta 24 >> $O/r3c_dir_ab.jsonl 2>>$O/r3c_dir_ab.err || { echo DIR_FAILED; exit 1; }
timeout -k 10 200 python -u benchmarks/kron_scale.py --scales 20,22,24 --queries 16 --alpha 50 --beta 24 >> $O/r3c_dir_ab.jsonl 2>>$O/r3c_dir_ab.err || { echo DIR_FAILED; exit 1; }
python3 -c "
import json
for l in open('$O/r3c_dir_ab.jsonl'):
    d=json.loads(l); print(d['graph'],d['direction'],d['alpha'],d['median_query_ms'],d['mean_query_ms'],d['mean_bottomup_levels'],d['mean_grid_levels'])"
