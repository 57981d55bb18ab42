#!/bin/bash
# per-kernel breakdown of the Mamba selective scan at config E scale (rocprofv3 --kernel-trace --stats)
set -e
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/scanprof
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/scan_bench.py --iters 3 "$@" > $OUT/bench.log 2>&1
python - $OUT <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f'{r["Name"][:70]:72s} n={r["Calls"]:>4s} avg={float(r["AverageNs"])/1e3:9.1f}us tot%={float(r["Percentage"]):5.1f}')
PY
grep "selective scan" $OUT/bench.log
