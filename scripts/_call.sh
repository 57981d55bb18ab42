set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
bash scripts/gpu.sh ab-env DNA_DDP_FORCE "0 1" 3
cp gpurun_out/ab.log gpurun_out/r06/ab_reducer_force.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_gpu_rccl.py > gpurun_out/r06/tests_rccl.log 2>&1
tail -3 gpurun_out/r06/tests_rccl.log
