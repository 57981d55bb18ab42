#!/bin/bash
# wgrad: hipBLASLt split-K (default) vs the persistent token-major kernel, bench shape.
set -o pipefail
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 300 python scripts/gemm_shapes.py --kinds wgrad --rounds 2 --iters 10 \
  --variants "base;hipw,DNA_WGRAD_IMPL=hip" > $O/wgrad.jsonl 2> $O/wgrad.err || { tail -20 $O/wgrad.err; exit 1; }
cat $O/wgrad.jsonl
