#!/bin/bash
# quick A/B: check + single-kernel timings under env variants (VAR=values list in $1, e.g. "DNA_GEMM_ABLATE=0 1 2")
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
L=gpurun_out/gemm_ab.log
: > $L
timeout -k 10 200 python scripts/gemm_bench.py --M 4096 --iters 2 >> $L 2>&1 | true
grep -q "CHECK PASS" $L || { cat $L; exit 1; }
VAR=${1%%=*}; VALS=${1#*=}
JOBS=${2:-"Wg:fwd Wwo:fwd Wqkv:fwd Wg:dgrad"}
for v in $VALS; do
  for job in $JOBS; do
    env $VAR=$v timeout -k 10 60 python scripts/gemm_bench.py --only $job --iters 20 2>&1 | grep -v amdgpu.ids | sed "s/^/$VAR=$v /" >> $L || exit 1
  done
done
cat $L
