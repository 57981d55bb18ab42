#!/bin/bash
# FlashAttention slot parity, Caduceus DDP (2 gloo ranks on one GPU), config E line, wgrad A/B.
set -o pipefail
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_flash_slot.py tests/test_ops_registry.py tests/test_gpu_caduceus_ddp.py -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert" $O/tests.txt | tail -70
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/caduceus_bench.py --steps 5 --warmup 2 --json $O/config_e.json > $O/config_e.txt 2>&1 || { tail -20 $O/config_e.txt; exit 1; }
cut -c1-400 $O/config_e.txt
timeout -k 10 300 python scripts/gemm_shapes.py --kinds wgrad --rounds 2 --iters 10 \
  --variants "base;hipw,DNA_WGRAD_IMPL=hip" > $O/wgrad.jsonl 2> $O/wgrad.err || { tail -20 $O/wgrad.err; exit 1; }
cat $O/wgrad.jsonl
