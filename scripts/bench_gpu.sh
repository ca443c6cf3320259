#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 python bench.py --no-resident --extra-graph "" > gpurun_out/bench_oneshot.json 2>> gpurun_out/bench.err
