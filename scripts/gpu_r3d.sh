#!/bin/bash
# FlashAttention slot parity + the wgrad A/B (hipBLASLt split-K vs the persistent kernel).
set -o pipefail
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_flash_slot.py tests/test_ops_registry.py -x -v --timeout 120 --timeout-method thread > $O/flash.txt 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert" $O/flash.txt | tail -60
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/gemm_shapes.py --kinds wgrad --rounds 2 --iters 10 \
  --variants "base;hipw,DNA_WGRAD_IMPL=hip" > $O/wgrad.jsonl 2> $O/wgrad.err || { tail -20 $O/wgrad.err; exit 1; }
cat $O/wgrad.jsonl
