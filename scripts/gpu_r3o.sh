#!/bin/bash
# FFT conv kernels specialised on compile-time sizes (N = 2^16..2^18) vs the generic ones.
set -o pipefail
O=gpurun_out/r3o
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_hyena.py tests/test_gpu_hyena_lm.py -q -x --timeout 300 --timeout-method thread > $O/fft_tests.log 2>&1 || { tail -30 $O/fft_tests.log; exit 1; }
tail -2 $O/fft_tests.log
for v in generic fixed generic2 fixed2; do
  case $v in generic*) E="DNA_FFT_GENERIC=1";; *) E="DNA_FFT_GENERIC=0";; esac
  env $E timeout -k 10 200 python scripts/fftconv_bench.py --dtype bf16,fp32 > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "== $v"; grep B= $O/bench_$v.log
done
