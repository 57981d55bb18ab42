#!/bin/bash
# Round 3 bundle: the DNABERT-2 bench under rocprof (+ data path) / PMC traffic / default bench,
# the config-E and config-D lines, attention-backward PMC (LDS bank conflicts).
set -o pipefail
ROUND=r03 BATCH=512 bash scripts/gpu_round_profile.sh || { tail -5 gpurun_out/r03/*.err; exit 1; }
cut -c1-300 gpurun_out/r03/bench.json
head -12 gpurun_out/r03/kernel_stats.md
cat gpurun_out/r03/roofline_agreement.md
O=gpurun_out/r03
timeout -k 10 300 python scripts/caduceus_bench.py --steps 5 --warmup 2 --json $O/config_e.json > $O/config_e.txt 2>&1 || { tail -5 $O/config_e.txt; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/cfge_stats -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/caduceus_bench.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$O/cfge_prof.txt 2>&1 || exit 1
python $GRAFT_REPO_ROOT/scripts/prof_summary.py $GRAFT_REPO_ROOT/$O/cfge_stats/run_kernel_stats.csv --steps 4 > $GRAFT_REPO_ROOT/$O/config_e_kernel_stats.md
cd $GRAFT_REPO_ROOT
head -8 $O/config_e_kernel_stats.md
