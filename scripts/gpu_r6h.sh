#!/bin/bash
# fused GeGLU-backward cost split: real kernel (0), no GeGLU math (64), no g loads (128), the
# plain-epilogue GEMM and the separate pair; dropout p = 0.1
set -o pipefail
O=gpurun_out/${TAG:-r6h}
mkdir -p $O
VARS=0,64,128 P=0.1 ROUNDS=2 timeout -k 10 200 python scripts/geglu_bwd_ab.py > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
