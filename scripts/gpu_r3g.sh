#!/bin/bash
# Config-D tests at L=65536, then PMC passes for the wgrad kernel vs the forward at Wo.
set -o pipefail
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_hyena_lm.py -x -v --timeout 200 --timeout-method thread > $O/hyena.txt 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert" $O/hyena.txt | tail -20
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_shape_pmc.sh r3g/pmc Wo:wgrad:DNA_WGRAD_IMPL=hip Wo:fwd:- Wo:wgrad:-
