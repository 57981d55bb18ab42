#!/bin/bash
# A/B at the bench shape: wgrad (hipBLASLt split-K vs the persistent token-major kernel, 8- and
# 10-slot LDS ring) and the forward / dgrad persistent GEMM (two-buffer vs ring); then the
# bench-shape GEMM parity tests (both ring settings) and the attention kernel tests.
set -o pipefail
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 300 python scripts/gemm_shapes.py --kinds wgrad --rounds 2 --iters 10 \
  --variants "base;hip8,DNA_WGRAD_IMPL=hip,DNA_WGRAD_RING=8;hip10,DNA_WGRAD_IMPL=hip,DNA_WGRAD_RING=10" > $O/wgrad.jsonl 2> $O/wgrad.err || { tail -20 $O/wgrad.err; exit 1; }
cat $O/wgrad.jsonl
timeout -k 10 300 python scripts/gemm_shapes.py --kinds fwd,dgrad --rounds 2 --iters 10 \
  --variants "base;ring,DNA_GEMM_RING=10" > $O/fwd.jsonl 2> $O/fwd.err || { tail -20 $O/fwd.err; exit 1; }
cat $O/fwd.jsonl
DNA_GEMM_RING=10 timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 200 --timeout-method thread -k "bench_shape or wgrad or ragged or gemm" > $O/tests.txt 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert" $O/tests.txt | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 200 --timeout-method thread -k "attention or bench_shape" > $O/attn.txt 2>&1
rc=$?
tail -3 $O/attn.txt
exit $rc
