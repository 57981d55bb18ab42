#!/bin/bash
# Config D: implicit-filter MLP as split-K batched products (DNA_HYENA_FILTER_SPLITK) -- test, A/B.
set -o pipefail
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hyena_lm.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in off on off2 on2; do
  case $v in off*) E="DNA_HYENA_FILTER_SPLITK=0";; *) E="DNA_HYENA_FILTER_SPLITK=1";; esac
  env $E timeout -k 10 300 python scripts/hyena_lm_bench.py --steps 5 > $O/cfgd_$v.log 2>&1 || { tail -20 $O/cfgd_$v.log; exit 1; }
  echo "== $v $(grep 'train step' $O/cfgd_$v.log | cut -c1-120)"
done
