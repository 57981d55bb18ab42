#!/bin/bash
# GeGLU-bwd fused GEMM variant check: geglu parity tests, then the bench's per-kernel line.
set -o pipefail
O=gpurun_out/${TAG:-r6c}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -k "geglu" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_new.log 2>&1 || { tail -40 $O/tests_new.log; exit 1; }
grep -E "passed|failed" $O/tests_new.log | tail -3
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
python -c "import json;d=json.load(open('$O/bench.json'));print({k:(v['avg_ms'],v.get('frac')) for k,v in d['kernels'].items()})"
