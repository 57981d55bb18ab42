#!/bin/bash
# GEMM: bias-initialised accumulators (DNA_GEMM_ABL=128) -- parity, shape A/B.
set -o pipefail
O=gpurun_out/r3z
mkdir -p $O
DNA_GEMM_ABL=128 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k "gemm or linear" > $O/test_bi.log 2>&1 || { tail -30 $O/test_bi.log; exit 1; }
tail -2 $O/test_bi.log
timeout -k 10 400 python scripts/gemm_shapes.py --kinds fwd,dgrad --rounds 3 --iters 10 \
  --variants "base;bi,DNA_GEMM_ABL=128" > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
