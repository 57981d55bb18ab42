#!/bin/bash
# even row-block split: bench-shape GEMM / GeGLU parity tests, then the bench line
set -o pipefail
O=gpurun_out/${TAG:-r6l}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -k "bench_shape or geglu or row_block or ragged" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
python -c "import json;d=json.load(open('$O/bench.json'));print(d['roofline']['frac'], {k:(v['avg_ms'],v.get('frac')) for k,v in d['kernels'].items()})"
