#!/bin/bash
# Attention backward packed-f32 tail (DNA_ATTN_BWD3_PK=1): parity, then A/B at the bench shape;
# config-D L=65536 tests.
set -o pipefail
O=gpurun_out/r3l
mkdir -p $O
DNA_ATTN_BWD3_PK=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k "attention" > $O/test_pk.log 2>&1 || { tail -30 $O/test_pk.log; exit 1; }
tail -2 $O/test_pk.log
for v in base pk sb; do
  case $v in base) E="";; pk) E="DNA_ATTN_BWD3_PK=1";; sb) E="DNA_ATTN_BWD3_SB=1";; esac
  env $E timeout -k 10 120 python scripts/attn_bench.py --b 512 --which bwd > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "== $v"; cat $O/bench_$v.log
done
env DNA_ATTN_BWD3_PK=1 timeout -k 10 120 python scripts/attn_bench.py --b 512 --which bwd > $O/bench_pk2.log 2>&1 && echo "== pk2" && cat $O/bench_pk2.log
timeout -k 10 120 python scripts/attn_bench.py --b 512 --which bwd > $O/bench_base2.log 2>&1 && echo "== base2" && cat $O/bench_base2.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_hyena_lm.py -k "65536" > $O/test_cfgd.log 2>&1 || { tail -30 $O/test_cfgd.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/test_cfgd.log | tail -5
