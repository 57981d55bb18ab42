#!/bin/bash
# Round 3, first GPU pass: GEMM kernels (incl. the ragged-M canary), the self-launched 2-rank
# bench (gloo rehearsal on one GPU), and a short default bench with the spawned data pipeline.
set -o pipefail
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread > $O/kernels.txt 2>&1 || { tail -30 $O/kernels.txt; exit 1; }
tail -3 $O/kernels.txt
DNA_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --batch 64 --steps 5 --warmup 2 --no-cpu-baseline --no-b64 > $O/bench_2rank.txt 2> $O/bench_2rank.err || { tail -30 $O/bench_2rank.err; exit 1; }
cat $O/bench_2rank.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-b64 > $O/bench.txt 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.txt
