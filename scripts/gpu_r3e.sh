#!/bin/bash
# wgrad A/B at the bench shape: hipBLASLt split-K vs the persistent token-major kernel.
set -o pipefail
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 300 python scripts/gemm_shapes.py --kinds wgrad --rounds 2 --iters 10 \
  --variants "base;hipw,DNA_WGRAD_IMPL=hip" > $O/wgrad.jsonl 2> $O/wgrad.err || { tail -20 $O/wgrad.err; exit 1; }
cat $O/wgrad.jsonl
