set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_gpu_kernels.py -k "geglu or dropout" tests/test_ops_registry.py > gpurun_out/r06/tests_keep.log 2>&1
tail -2 gpurun_out/r06/tests_keep.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_gpu_model.py > gpurun_out/r06/tests_model.log 2>&1
tail -2 gpurun_out/r06/tests_model.log
bash scripts/gpu.sh ab-env DNA_GEMM_ABL "0 256" 3
cp gpurun_out/ab.log gpurun_out/r06/ab_geglu_keep_ahead.txt
