#!/bin/bash
# The hand-written weight gradient as the default: per-shape A/B (incl. the immediate-offset
# reads), then interleaved bench A/B against hipBLASLt, then the model / trainer GPU tests.
set -o pipefail
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 300 python scripts/gemm_shapes.py --kinds wgrad --rounds 2 --iters 10 \
  --variants "torch,DNA_WGRAD_IMPL=torch;hip,DNA_WGRAD_IMPL=hip;hipnoimm,DNA_WGRAD_IMPL=hip,DNA_WGRAD_IMM=0" > $O/wgrad.jsonl 2> $O/wgrad.err || { tail -20 $O/wgrad.err; exit 1; }
cat $O/wgrad.jsonl
for impl in hip torch hip torch; do
  echo "wgrad=$impl" >> $O/ab_bench.txt
  DNA_WGRAD_IMPL=$impl timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-b64 --no-cpu-baseline --no-data-pipeline >> $O/ab_bench.txt 2>> $O/ab_bench.err || exit 1
done
python - <<'PY'
import json
lines=open("gpurun_out/r3h/ab_bench.txt").read().splitlines()
for tag, l in zip(lines[0::2], lines[1::2]):
    d=json.loads(l); print(tag, d["value"], d["ms_per_step"], {k: (v["avg_ms"], v.get("frac")) for k, v in d["kernels"].items() if "gemm" in k})
PY
for v in 0 2 0 2; do
  echo "attn_fwd=$v $(DNA_ATTN_FWD=$v timeout -k 10 120 python scripts/attn_bench.py --b 512 --which fwd 2>/dev/null | tail -1)" >> $O/ab_attn.txt || exit 1
done
cat $O/ab_attn.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_trainer.py tests/test_gpu_kernels.py -x -v --timeout 300 --timeout-method thread -k "not bench_shape" > $O/tests.txt 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert" $O/tests.txt | tail -40
exit $rc
