#!/bin/bash
# FFT conv blocks of 4096 points / 256 threads (FFT_LOG_PTS=12 library) vs 8192 / 512: parity, bench.
set -o pipefail
O=gpurun_out/r4f
mkdir -p $O
L12=$GRAFT_REPO_ROOT/dna_amd/lib_ab/libdna_amd_pts12.so
DNA_AMD_LIB=$L12 timeout -k 10 400 python -u -m pytest tests/test_gpu_hyena.py -q -x --timeout 300 --timeout-method thread > $O/tests12.log 2>&1 || { tail -30 $O/tests12.log; exit 1; }
tail -1 $O/tests12.log
for v in p13 p12 p13b p12b; do
  case $v in p12*) export DNA_AMD_LIB=$L12;; *) unset DNA_AMD_LIB;; esac
  timeout -k 10 200 python scripts/fftconv_bench.py --dtype bf16,fp32 > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "== $v"; grep B= $O/bench_$v.log | cut -c1-200
done
