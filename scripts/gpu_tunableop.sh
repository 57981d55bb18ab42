# GEMM probe with PyTorch TunableOp tuning (hipBLASLt + rocBLAS solution search per shape)
set -e
mkdir -p gpurun_out/tunable
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1
export PYTORCH_TUNABLEOP_FILENAME=$GRAFT_REPO_ROOT/gpurun_out/tunable/tunableop_results%d.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=300 PYTORCH_TUNABLEOP_ROCBLAS_ENABLED=1
timeout -k 10 900 python scripts/gemm_probe.py 65536 > gpurun_out/tunable/probe_tuning.log 2>&1
export PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_VERBOSE=0
timeout -k 10 300 python scripts/gemm_probe.py 65536 > gpurun_out/tunable/probe_tuned.log 2>&1
