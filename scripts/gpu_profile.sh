# rocprofv3 kernel trace + stats of a short bench run; summary into gpurun_out/prof
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps ${STEPS:-10} --warmup 3 --batch ${BATCH:-128} --no-cpu-baseline --no-kernel-timing > $OUT/bench.json 2> $OUT/bench.err
python $GRAFT_REPO_ROOT/scripts/prof_summary.py $OUT/run_kernel_stats.csv --steps $(( ${STEPS:-10} + 3 )) > $OUT/summary.md
