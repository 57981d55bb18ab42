#!/bin/bash
# Lean persistent GEMM schedule (DNA_GEMM_SCHED=2) vs default: parity tests under it, per-shape A/B.
set -o pipefail
O=gpurun_out/${TAG:-r5c}
mkdir -p $O
DNA_GEMM_SCHED=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "gemm" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python scripts/gemm_shapes.py --kinds fwd,dgrad --rounds 3 --iters 10 \
  --variants "${VARIANTS:-base;sch2,DNA_GEMM_SCHED=2}" > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
