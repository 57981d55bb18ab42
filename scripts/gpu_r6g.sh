#!/bin/bash
# fused GeGLU-backward cost split: dropout on / off vs the plain-epilogue GEMM and the pair
set -o pipefail
O=gpurun_out/${TAG:-r6g}
mkdir -p $O
P=0.1 ROUNDS=2 timeout -k 10 200 python scripts/geglu_bwd_ab.py > $O/ab_p01.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
P=0.0 ROUNDS=2 timeout -k 10 200 python scripts/geglu_bwd_ab.py > $O/ab_p0.jsonl 2>> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab_p01.jsonl $O/ab_p0.jsonl
