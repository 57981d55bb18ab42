#!/bin/bash
# Attention A/B on the GPU box: parity tests of the attention kernels, then the micro-bench at
# the bench shape for the default kernels, the 4-wave v2 backward, and the v1 kernels.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "attention" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/attn_tests.log 2>&1
timeout -k 10 120 python scripts/attn_bench.py --b 256 ${ATTN_ARGS:-} > gpurun_out/attn_bench.log 2>&1
DNA_ATTN_BWD_NW=4 timeout -k 10 120 python scripts/attn_bench.py --b 256 --which bwd >> gpurun_out/attn_bench.log 2>&1
DNA_ATTN_FWD=1 DNA_ATTN_BWD=1 timeout -k 10 120 python scripts/attn_bench.py --b 256 >> gpurun_out/attn_bench.log 2>&1
cat gpurun_out/attn_bench.log
