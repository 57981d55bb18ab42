#!/bin/bash
# Round measurement bundle (GPU box): rocprofv3 --kernel-trace --stats of the bench command (with
# train.py's data path measured before GPU init, its DataLoader workers included), FETCH_SIZE and
# WRITE_SIZE --pmc passes (separate runs, kernel-trace only) -> traffic.json, the rocprof-vs-HIP
# event agreement table, then the default bench line (which reads profiles/<round>/traffic.json).
# Outputs under gpurun_out/<round>/; copy them into profiles/<round>/ afterwards.
set -e
R=${ROUND:-r03}
BATCH=${BATCH:-512}
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/$R
mkdir -p $OUT $ROOT/profiles/$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python $ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-b64 --batch $BATCH > $OUT/stats_bench.json 2> $OUT/stats_bench.err
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python $ROOT/bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-b64 --no-data-pipeline --batch $BATCH > $OUT/fetch_bench.json 2> $OUT/fetch_bench.err
timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python $ROOT/bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-b64 --no-data-pipeline --batch $BATCH > $OUT/write_bench.json 2> $OUT/write_bench.err
python $ROOT/scripts/traffic_from_pmc.py $OUT/fetch $OUT/write $OUT/traffic.json $BATCH $OUT/fetch_bench.json > /dev/null
cp $OUT/traffic.json $ROOT/profiles/$R/traffic.json
python $ROOT/scripts/prof_summary.py $OUT/stats/run_kernel_stats.csv --steps 13 > $OUT/kernel_stats.md
python $ROOT/scripts/roofline_agree.py $OUT/stats/run_kernel_stats.csv $OUT/stats_bench.json 13 > $OUT/roofline_agreement.md
cd $ROOT
timeout -k 10 600 python bench.py --batch $BATCH > $OUT/bench.json 2> $OUT/bench.err
rm -rf $OUT/fetch $OUT/write
