#!/bin/bash
# GEMM/wgrad parity tests + per-shape A/B of the default (lean) schedule against DNA_GEMM_SCHED=0.
set -o pipefail
O=gpurun_out/${TAG:-r5f}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "gemm or wgrad" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python scripts/gemm_shapes.py --kinds ${KINDS:-fwd,dgrad,wgrad} --rounds 3 --iters 10 \
  --variants "${VARIANTS:-sch2;sch0,DNA_GEMM_SCHED=0}" > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
