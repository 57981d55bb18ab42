#!/bin/bash
# Tune every GEMM of the bench step with PyTorch TunableOp (all hipBLASLt + rocBLAS solutions per
# shape, timed on the box) and keep the winners in gpurun_out/tune/tunableop_results.csv.
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/tune
mkdir -p $OUT
BATCH=${BATCH:-256}
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
PYTORCH_TUNABLEOP_FILENAME=$OUT/tunableop_results.csv \
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=60 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=10 \
  timeout -k 10 900 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --batch $BATCH \
  > $OUT/tune_bench.json 2> $OUT/tune.log
ls -la $OUT; wc -l $OUT/tunableop_results*.csv
