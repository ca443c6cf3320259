mkdir -p gpurun_out
timeout -k 10 300 python3 benchmarks/pair_latency.py --graph kron:22:16:1 --pairs 64 --reps 5 > gpurun_out/r5_kron22_pairs_probe.jsonl 2> gpurun_out/pl.err || exit 1
python3 -c "
import json
rs=[json.loads(l) for l in open('gpurun_out/r5_kron22_pairs_probe.jsonl')]
h=[r for r in rs if r['probe_hit']][:2]; m=[r for r in rs if r['handoff']][:1]
print(' '.join(f\"{r['src']}:{r['dst']}\" for r in h+m))" > gpurun_out/stamp_pairs.txt || exit 1
for p in $(cat gpurun_out/stamp_pairs.txt); do
  BIBFS_STAMP=1 timeout -k 10 120 ./build/bin/bibfs_hip kron:22:16:1 ${p%%:*} ${p##*:} --trace --repeat 4 --verify >> gpurun_out/r5_kron22_probe_stamps.txt 2>&1 || exit 1
done
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5probe_bench.json 2> gpurun_out/r5probe_bench.err
