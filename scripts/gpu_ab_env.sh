#!/bin/bash
# Interleaved A/B of an environment switch on the bench step (GPU box):
#   AB_VAR=NAME AB_A=val AB_B=val bash scripts/gpu_ab_env.sh   (or AB_VALS="v1 v2 v3")
# runs the GPU test suite once, then bench.py alternately with NAME=A / NAME=B (2 each).
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests.log 2>&1
for rep in 1 2; do
  for v in ${AB_VALS:-$AB_A $AB_B}; do
    env $AB_VAR=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-b64 > gpurun_out/ab.json 2>gpurun_out/ab.err
    echo "$AB_VAR=$v $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'], {k: round(v['avg_ms'],3) for k,v in d['kernels'].items()})")"
  done
done > gpurun_out/ab.log
cat gpurun_out/ab.log
