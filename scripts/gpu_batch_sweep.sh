#!/bin/bash
# per-GPU batch sweep of the headline bench (plus the default bench line first)
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 500 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
: > gpurun_out/sweep.jsonl
for b in 32 64 128 256; do
  timeout -k 10 400 python bench.py --batch $b --steps 20 --warmup 5 --no-cpu-baseline >> gpurun_out/sweep.jsonl 2> gpurun_out/sweep_b$b.err
done
