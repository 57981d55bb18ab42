#!/bin/bash
# FFT long conv chunked for Infinity-Cache residency (DNA_FFT_CHUNK_MB): parity, then A/B.
set -o pipefail
O=gpurun_out/r3n
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_hyena.py -q -x --timeout 200 --timeout-method thread > $O/fft_tests.log 2>&1 || { tail -30 $O/fft_tests.log; exit 1; }
tail -2 $O/fft_tests.log
DNA_FFT_CHUNK_MB=8 timeout -k 10 400 python -u -m pytest tests/test_gpu_hyena.py -q -x --timeout 200 --timeout-method thread > $O/fft_tests8.log 2>&1 || { tail -30 $O/fft_tests8.log; exit 1; }
tail -2 $O/fft_tests8.log
for mb in 0 64 32 128 16; do
  DNA_FFT_CHUNK_MB=$mb timeout -k 10 200 python scripts/fftconv_bench.py --dtype bf16,fp32 > $O/bench_$mb.log 2>&1 || { tail -20 $O/bench_$mb.log; exit 1; }
  echo "== chunk $mb MB"; grep B= $O/bench_$mb.log
done
