#!/bin/bash
# Early-stage schedule (DNA_GEMM_SCHED=3: each LDS-DMA stage issued before the previous phase's
# MFMAs, one more phase of slack for the epilogue stores): GEMM parity tests, per-shape A/B.
set -o pipefail
O=gpurun_out/${TAG:-r5j}
mkdir -p $O
DNA_GEMM_SCHED=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "gemm" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python scripts/gemm_shapes.py --kinds fwd,dgrad --rounds 3 --iters 10 \
  --variants "sch2;sch3,DNA_GEMM_SCHED=3" > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
