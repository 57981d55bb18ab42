set -e
cd $GRAFT_REPO_ROOT
bash scripts/gpu.sh round r06
cat gpurun_out/r06/bench.json | cut -c1-300
