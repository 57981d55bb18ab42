#!/bin/bash
# GeGLU forward fused into the gated_layers GEMM epilogue (lean persistent kernel): kernel + model
# parity tests, then the bench with and without the fusion.
set -o pipefail
O=gpurun_out/${TAG:-r5i}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -k "gemm or geglu or wgrad or model or bf16 or grads or forward" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in fused unfused fused2; do
  case $v in unfused) export DNA_GEGLU_FUSED=0;; *) unset DNA_GEGLU_FUSED;; esac
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-data-pipeline > $O/bench_$v.json 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  echo "== $v"; python -c "import json;d=json.load(open('$O/bench_$v.json'));print(d['value'],d['ms_per_step'],{k:(v['avg_ms'],v.get('frac')) for k,v in d['kernels'].items()})"
done
