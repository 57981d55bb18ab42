#!/bin/bash
# Row-blocked GEMM + HipLinear tests and the full GPU suite; batch A/B; the round measurement
# bundle at the default per-GPU batch (512); config-D projection A/B with a rocprof summary.
set -o pipefail
O=gpurun_out/s8
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_hyena_lm.py -x -q --timeout 120 --timeout-method thread > $O/new_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || exit 1
for b in 256 512; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-b64 --no-cpu-baseline --no-data-pipeline --batch $b >> $O/ab_batch.jsonl 2>> $O/ab_batch.err || exit 1
done
DNA_HYENA_TORCH_LINEAR=1 timeout -k 10 120 python scripts/hyena_lm_bench.py > $O/cfgd_torchlinear.txt 2>&1 || exit 1
timeout -k 10 120 python scripts/hyena_lm_bench.py > $O/cfgd_hiplinear.txt 2>&1 || exit 1
ROUND=r02b512 BATCH=512 timeout -k 10 700 bash scripts/gpu_round_profile.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/cfgd_stats -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/hyena_lm_bench.py > $GRAFT_REPO_ROOT/$O/cfgd_prof.txt 2>&1 || exit 1
