#!/bin/bash
# GeGLU-backward GEMM variants (VARS): parity, then kernel A/B
set -o pipefail
O=gpurun_out/${TAG:-r6i}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "geglu_dgrad" -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
VARS=0,256 P=0.1 ROUNDS=3 timeout -k 10 200 python scripts/geglu_bwd_ab.py > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
