#!/bin/bash
# Hyena op kernels templated on the operator order vs the round-2 kernels (old library), bf16 at
# config-D scale through hyena_lm_bench (per-op HIP-event times).
set -o pipefail
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_hyena.py -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in new old new2 old2; do
  case $v in old*) export DNA_AMD_LIB=$GRAFT_REPO_ROOT/dna_amd/lib_ab/libdna_amd_old.so;; *) unset DNA_AMD_LIB;; esac
  timeout -k 10 300 python scripts/hyena_lm_bench.py --steps 5 > $O/cfgd_$v.log 2>&1 || { tail -20 $O/cfgd_$v.log; exit 1; }
  echo "== $v $(grep 'train step' $O/cfgd_$v.log | grep -o '[0-9.]* seq/s\|hyena_[a-z_]* [0-9.]* ms' | tr '\n' ' ')"
done
