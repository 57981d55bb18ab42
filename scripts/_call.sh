set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
set +e
PYTHONFAULTHANDLER=1 DNA_DDP_FORCE=1 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-b64 --no-data-pipeline > gpurun_out/r06/force.json 2> gpurun_out/r06/force.err
echo "force rc=$?"
set -e
DNA_DIST_BACKEND=gloo timeout -k 10 200 python scripts/wire_error.py --ranks 4 --batch 8 > gpurun_out/r06/wire4.json 2> gpurun_out/r06/wire4.err
cat gpurun_out/r06/wire4.json
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_gpu_ddp_wire.py tests/test_gpu_rccl.py tests/test_gpu_trainer.py tests/test_train_cli.py \
  "tests/test_gpu_kernels.py::test_dropout_mask_consistent_fwd_bwd" "tests/test_gpu_caduceus.py::test_caduceus_odd_d_inner_autocast" > gpurun_out/r06/tests_dist.log 2>&1
tail -3 gpurun_out/r06/tests_dist.log
