#!/bin/bash
# shortconv_bwd rewrite: parity, then HyenaOperator per-kernel stats new vs old library.
set -o pipefail
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_hyena.py -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cd /tmp && export TMPDIR=/tmp
for v in new old; do
  if [ $v = old ]; then export DNA_AMD_LIB=$GRAFT_REPO_ROOT/dna_amd/lib_ab/libdna_amd_old.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_$v -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/hyena_op_bench.py --iters 5 --B 2 > $GRAFT_REPO_ROOT/$O/bench_$v.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/bench_$v.log; exit 1; }
  echo "== $v"; grep HyenaOperator $GRAFT_REPO_ROOT/$O/bench_$v.log
  python - $GRAFT_REPO_ROOT/$O/prof_$v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f))):
    if "hyop" in r["Name"]:
        print(f'{r["Name"][:70]:72s} n={r["Calls"]:>4s} avg={float(r["AverageNs"])/1e3:9.1f}us')
PY
done
