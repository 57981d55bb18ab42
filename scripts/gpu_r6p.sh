#!/bin/bash
# vector cross-entropy kernels: CE / model parity tests, bench, rocprof rows
set -o pipefail
O=gpurun_out/${TAG:-r6p}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_ops_registry.py -k "cross_entropy or xent or golden or reference or loss or task" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-b64 --no-data-pipeline > /dev/null 2>&1 || exit 1
grep -i "xent" $GRAFT_REPO_ROOT/$O/prof/run_kernel_stats.csv | cut -c1-160
