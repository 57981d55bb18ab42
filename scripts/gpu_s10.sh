#!/bin/bash
# Weight-gradient split-K cap A/B at the default per-GPU batch (512), interleaved.
set -o pipefail
O=gpurun_out/s10
mkdir -p $O
for s in 64 32 16 64 32 16; do
  echo "max_splits=$s" >> $O/ab_splits.txt
  DNA_WGRAD_MAX_SPLITS=$s timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-b64 --no-cpu-baseline --no-data-pipeline >> $O/ab_splits.txt 2>> $O/ab_splits.err || exit 1
done
