#!/bin/bash
# Three-stage phase-1 attention backward (DNA_ATTN_BWD3_P3=1): parity, then A/B at the bench shape.
set -o pipefail
O=gpurun_out/r3y
mkdir -p $O
DNA_ATTN_BWD3_P3=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k "attention" > $O/test_p3.log 2>&1 || { tail -30 $O/test_p3.log; exit 1; }
tail -2 $O/test_p3.log
for v in base p3 base2 p32; do
  case $v in base*) E="";; p3*) E="DNA_ATTN_BWD3_P3=1";; esac
  env $E timeout -k 10 120 python scripts/attn_bench.py --b 512 --which bwd > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "== $v $(grep attn_bwd $O/bench_$v.log)"
done
