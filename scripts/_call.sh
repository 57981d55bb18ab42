set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_gpu_ddp_wire.py tests/test_gpu_rccl.py tests/test_gpu_trainer.py tests/test_train_cli.py \
  "tests/test_gpu_kernels.py::test_dropout_mask_consistent_fwd_bwd" tests/test_gpu_caduceus.py tests/test_gpu_caduceus_ddp.py \
  tests/test_gpu_hyena_lm.py > gpurun_out/r06/tests_dist.log 2>&1
tail -3 gpurun_out/r06/tests_dist.log
for r in 1 2; do for v in 3 4; do
  DNA_FFT_RB_BLOCKS=$v timeout -k 10 120 python scripts/fftconv_bench.py --B 2 --D 256 --L 65536 --dtype bf16 --bidirectional 1 --iters 20 > gpurun_out/r06/fft_rb$v.txt 2>&1
  echo "RB=$v $(grep -i bwd gpurun_out/r06/fft_rb$v.txt | head -3 | tr '\n' ' ')" | tee -a gpurun_out/r06/fft_rb_ab.txt
done; done
bash scripts/gpu.sh ab-env DNA_DDP_FORCE "0 1" 3
cp gpurun_out/ab.log gpurun_out/r06/ab_reducer_force.txt
