#!/bin/bash
# Forward GEMM main-loop ablations (timing only): staging / LDS reads / barriers removed.
set -o pipefail
O=gpurun_out/r3j
mkdir -p $O
timeout -k 10 300 python scripts/gemm_shapes.py --kinds fwd --only Wwo,Wo,Wg --rounds 2 --iters 10 \
  --variants "base;noBread,DNA_GEMM_ABL=16;noBstage,DNA_GEMM_ABL=32;noB,DNA_GEMM_ABL=8" > $O/abl.jsonl 2> $O/abl.err || { tail -20 $O/abl.err; exit 1; }
cat $O/abl.jsonl
