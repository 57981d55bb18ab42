#!/bin/bash
# Config D (HyenaDNA-small, L=65536) bench line + rocprof summary after the FFT / shortconv changes.
set -o pipefail
O=gpurun_out/r3r
mkdir -p $O
timeout -k 10 400 python scripts/hyena_lm_bench.py --steps 5 > $O/cfgd.log 2>&1 || { tail -30 $O/cfgd.log; exit 1; }
grep -v "^{" $O/cfgd.log | tail -3; grep "^{" $O/cfgd.log > $O/config_d.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/hyena_lm_bench.py --steps 3 > $GRAFT_REPO_ROOT/$O/cfgd_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/cfgd_prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && python scripts/prof_summary.py $O/prof/run_kernel_stats.csv --top 25 > $O/config_d_kernel_stats.md && head -30 $O/config_d_kernel_stats.md
