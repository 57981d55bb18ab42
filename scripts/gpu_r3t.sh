#!/bin/bash
# GEMM: use-ordered fragment reads with counted LDS waits (DNA_GEMM_ABL=64) -- parity, shape A/B.
set -o pipefail
O=gpurun_out/r3t
mkdir -p $O
DNA_GEMM_ABL=64 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k "gemm or linear" > $O/test_fl.log 2>&1 || { tail -30 $O/test_fl.log; exit 1; }
tail -2 $O/test_fl.log
timeout -k 10 400 python scripts/gemm_shapes.py --kinds fwd,dgrad --rounds 3 --iters 10 \
  --variants "base;fl,DNA_GEMM_ABL=64" > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
