#!/bin/bash
# per-kernel breakdown of the FFT long conv at config D (rocprofv3 --kernel-trace --stats),
# then PMC passes (separate runs) on the same command
set -e
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/fftprof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
CMD="python $ROOT/scripts/fftconv_bench.py --dtype fp32 --iters 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- $CMD > $OUT/bench.log 2>&1
python $ROOT/scripts/prof_summary.py $OUT/run_kernel_stats.csv --top 20 > $OUT/summary.md
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set -d $OUT/col_fwd_$i -o run --output-format csv -- $CMD > $OUT/pmc$i.log 2>&1 || echo "pmc $i failed" >> $OUT/errors.txt
done
python $ROOT/scripts/pmc_table.py $OUT --kernel "col_fwd_kernel<float, 17>" > $OUT/pmc_colfwd.txt 2>&1 || true
python $ROOT/scripts/pmc_table.py $OUT --kernel "row_kernel<1, 17>" > $OUT/pmc_row.txt 2>&1 || true
python $ROOT/scripts/pmc_table.py $OUT --kernel "col_inv_kernel<float, 0, 17>" > $OUT/pmc_colinv.txt 2>&1 || true
