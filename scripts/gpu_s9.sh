#!/bin/bash
# Caduceus: Mamba out_proj on the persistent MFMA GEMM (A/B), full GPU suite.
set -o pipefail
O=gpurun_out/s9
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || exit 1
DNA_HYENA_TORCH_LINEAR=1 timeout -k 10 150 python scripts/caduceus_bench.py > $O/cfge_torchlinear.txt 2>&1 || exit 1
timeout -k 10 150 python scripts/caduceus_bench.py > $O/cfge_hiplinear.txt 2>&1 || exit 1
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
