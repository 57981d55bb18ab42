#!/bin/bash
# Direct weight operand (DNA_GEMM_BD): GEMM parity under BD=2, then fwd / dgrad shape A/B.
set -o pipefail
O=gpurun_out/r3k
mkdir -p $O
DNA_GEMM_BD=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k "gemm or linear" > $O/test_bd.log 2>&1 || { tail -30 $O/test_bd.log; exit 1; }
tail -3 $O/test_bd.log
timeout -k 10 400 python scripts/gemm_shapes.py --kinds fwd,dgrad --rounds 2 --iters 10 \
  --variants "base;bd1,DNA_GEMM_BD=1;bd2,DNA_GEMM_BD=2" > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
