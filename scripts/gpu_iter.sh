# generic iteration: kernel tests, GEMM probe, bench (each step time-limited, stop on failure)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -q -m gpu --timeout 300 -p no:cacheprovider -x > gpurun_out/tests.log 2>&1
if [ "${PROBE:-0}" = "1" ]; then timeout -k 10 300 python scripts/gemm_probe.py 65536 > gpurun_out/gemm_probe.log 2>&1; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --batch ${BATCH:-128} ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
