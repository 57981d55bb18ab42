#!/bin/bash
# Per-GPU batch A/B (256 vs 512, interleaved on one box), then the round measurement bundle at 512.
set -o pipefail
O=gpurun_out/s5
mkdir -p $O
for b in 256 512 256 512; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-b64 --no-cpu-baseline --no-data-pipeline --batch $b >> $O/ab_batch.jsonl 2>> $O/ab_batch.err || exit 1
done
ROUND=r02b512 BATCH=512 timeout -k 10 900 bash scripts/gpu_round_profile.sh || exit 1
