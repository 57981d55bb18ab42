set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/ > gpurun_out/r06/gpu_suite_full.txt 2>&1
tail -2 gpurun_out/r06/gpu_suite_full.txt
