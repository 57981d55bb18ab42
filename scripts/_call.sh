set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_gpu_kernels.py -k "layernorm or ln_bwd or geglu" tests/test_gpu_model.py > gpurun_out/r06/tests_ln.log 2>&1
tail -3 gpurun_out/r06/tests_ln.log
bash scripts/gpu.sh ab-tree "main base" 3 20
