#!/bin/bash
# Weight-gradient side stream A/B at the default per-GPU batch (512), interleaved.
set -o pipefail
O=gpurun_out/s11
mkdir -p $O
for s in 0 1 0 1; do
  echo "wgrad_stream=$s" >> $O/ab_stream.txt
  DNA_WGRAD_STREAM=$s timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-b64 --no-cpu-baseline --no-data-pipeline >> $O/ab_stream.txt 2>> $O/ab_stream.err || exit 1
done
