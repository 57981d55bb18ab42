#!/bin/bash
# Philox A/B: the library built with mul_hi/mul_lo pairs (DNA_AMD_LIB=dna_amd/lib/ab/...) vs the
# 64-bit-product build (default), interleaved bench runs; dropout-bearing kernels compared.
set -o pipefail
O=gpurun_out/${TAG:-r6f}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "dropout or geglu or ln" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  DNA_AMD_LIB=$PWD/dna_amd/lib/ab/libdna_amd_philox_old.so timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-cpu-baseline --no-b64 --no-data-pipeline > $O/old_$i.json 2> $O/old_$i.err || { tail -20 $O/old_$i.err; exit 1; }
  timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-cpu-baseline --no-b64 --no-data-pipeline > $O/new_$i.json 2> $O/new_$i.err || { tail -20 $O/new_$i.err; exit 1; }
done
for f in $O/old_*.json $O/new_*.json; do python -c "import json,sys;d=json.load(open('$f'));print('$f', d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items() if k in ('gemm_geglu','gemm_geglu_bwd','ln_fwd','ln_bwd')})"; done
