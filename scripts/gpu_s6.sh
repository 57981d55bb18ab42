#!/bin/bash
# HipLinear tests, full GPU suite, config-D projection A/B (torch Linear vs the MFMA GEMM).
set -o pipefail
O=gpurun_out/s6
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_hyena_lm.py -x -q --timeout 100 --timeout-method thread > $O/hyena_test.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || exit 1
DNA_HYENA_TORCH_LINEAR=1 timeout -k 10 120 python scripts/hyena_lm_bench.py > $O/cfgd_torchlinear.txt 2>&1 || exit 1
timeout -k 10 120 python scripts/hyena_lm_bench.py > $O/cfgd_hiplinear.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/cfgd_stats -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/hyena_lm_bench.py > $GRAFT_REPO_ROOT/$O/cfgd_prof.txt 2>&1 || exit 1
