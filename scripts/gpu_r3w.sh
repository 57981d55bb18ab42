#!/bin/bash
# Bisect which earlier GPU test file makes test_geglu_row_unrolled_bf16[16387] fail in the suite.
set -o pipefail
O=gpurun_out/r3w
mkdir -p $O
T="tests/test_gpu_kernels.py::test_geglu_row_unrolled_bf16"
i=0
for pre in tests/test_gpu_caduceus.py tests/test_gpu_caduceus_ddp.py tests/test_gpu_config_e.py tests/test_gpu_flash_slot.py "tests/test_gpu_hyena.py tests/test_gpu_hyena_lm.py"; do
  i=$((i+1))
  timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider $pre "$T" > $O/b$i.log 2>&1
  echo "== $pre: $(tail -1 $O/b$i.log)"
done
