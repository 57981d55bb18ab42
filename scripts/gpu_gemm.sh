#!/bin/bash
# GEMM correctness + timing vs hipBLASLt on the GPU box.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python scripts/gemm_bench.py "$@" > gpurun_out/gemm_bench.log 2>&1
rc=$?
cat gpurun_out/gemm_bench.log
exit $rc
