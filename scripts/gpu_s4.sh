#!/bin/bash
# Session check bundle: new norm tests, full GPU suite, smoke, a short bench, config-D LayerNorm
# and config-E RMSNorm A/Bs, a b=512 bench.
set -o pipefail
O=gpurun_out/s4
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_hyena_lm.py tests/test_gpu_caduceus.py -x -q --timeout 100 --timeout-method thread > $O/norm_test.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 30 --warmup 10 --no-b64 --no-cpu-baseline --no-data-pipeline > $O/bench.json 2> $O/bench.err || exit 1
DNA_HYENA_TORCH_LN=1 timeout -k 10 120 python scripts/hyena_lm_bench.py > $O/cfgd_torchln.txt 2>&1 || exit 1
timeout -k 10 120 python scripts/hyena_lm_bench.py > $O/cfgd_hipln.txt 2>&1 || exit 1
DNA_CADUCEUS_TORCH_NORM=1 timeout -k 10 120 python scripts/caduceus_bench.py > $O/cfge_torchnorm.txt 2>&1 || exit 1
timeout -k 10 120 python scripts/caduceus_bench.py > $O/cfge_hipnorm.txt 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-b64 --no-cpu-baseline --no-data-pipeline --batch 512 > $O/bench_b512.json 2> $O/bench_b512.err || exit 1
