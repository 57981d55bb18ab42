#!/bin/bash
# GEMM per-shape timing at the bench shape: unit order / group-size variants vs hipBLASLt.
set -o pipefail
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 500 python scripts/gemm_shapes.py --torch --rounds 2 --iters 10 \
  --variants "base;xcd8,DNA_GEMM_ORDER=1,DNA_GEMM_GM=8;xcd16,DNA_GEMM_ORDER=1,DNA_GEMM_GM=16;xcd4,DNA_GEMM_ORDER=1,DNA_GEMM_GM=4;gm16,DNA_GEMM_GM=16" \
  > $O/shapes.jsonl 2> $O/shapes.err || { tail -20 $O/shapes.err; exit 1; }
cat $O/shapes.jsonl
