#!/bin/bash
# FFT long conv at config D: rocprofv3 --stats + separate FETCH_SIZE / WRITE_SIZE --pmc passes
set -e
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/fftr01
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
CMD="python $ROOT/scripts/fftconv_bench.py --dtype fp32 --iters 3"
timeout -k 10 300 $CMD > $OUT/bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- $CMD > $OUT/stats.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $CMD > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $CMD > $OUT/write.log 2>&1
python $ROOT/scripts/prof_summary.py $OUT/stats/run_kernel_stats.csv --top 25 > $OUT/kernel_stats.md
python $ROOT/scripts/fft_traffic.py $OUT/fetch $OUT/write $OUT/stats/run_kernel_stats.csv > $OUT/traffic.md
rm -rf $OUT/fetch $OUT/write
