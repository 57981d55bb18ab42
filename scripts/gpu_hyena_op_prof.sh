#!/bin/bash
# per-kernel breakdown of one HyenaOperator layer fwd+bwd at config-D scale
set -e
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/hyenaprof
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/hyena_op_bench.py --iters 3 "$@" > $OUT/bench.log 2>&1
python - $OUT <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:25]:
    print(f'{r["Name"][:90]:92s} n={r["Calls"]:>4s} avg={float(r["AverageNs"])/1e3:9.1f}us tot%={float(r["Percentage"]):5.1f}')
PY
grep "HyenaOperator" $OUT/bench.log
