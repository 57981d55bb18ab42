# generic iteration: GPU tests, smoke, optional GEMM probe, bench (each step time-limited)
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -q -m gpu --timeout 400 -p no:cacheprovider -x > gpurun_out/tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
if [ "${PROBE:-0}" = "1" ]; then timeout -k 10 300 python scripts/gemm_probe.py 65536 > gpurun_out/gemm_probe.log 2>&1; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --batch ${BATCH:-128} ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
