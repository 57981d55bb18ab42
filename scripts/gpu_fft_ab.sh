#!/bin/bash
# FFT long-conv check on the GPU box: parity tests, then the config-D micro-bench.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_hyena.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/fft_tests.log 2>&1
timeout -k 10 300 python scripts/fftconv_bench.py --dtype fp32,bf16 > gpurun_out/fft_bench.log 2>&1
cat gpurun_out/fft_bench.log
