#!/bin/bash
# Lean schedule as the default: kernel + model GPU tests, per-shape A/B (fwd/dgrad/wgrad) vs
# DNA_GEMM_SCHED=0, then the default bench.
set -o pipefail
O=gpurun_out/${TAG:-r5e}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python scripts/gemm_shapes.py --kinds fwd,dgrad,wgrad --rounds 3 --iters 10 \
  --variants "sch2;sch0,DNA_GEMM_SCHED=0" > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
