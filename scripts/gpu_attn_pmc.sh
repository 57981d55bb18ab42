# attention micro-bench + PMC counter passes (separate --pmc runs, kernel-trace only)
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/attn
mkdir -p $OUT
timeout -k 10 120 python $GRAFT_REPO_ROOT/scripts/attn_bench.py > $OUT/bench.txt 2>&1
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc $set -d $OUT/pmc$i -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/attn_bench.py --iters 3 > $OUT/pmc$i.log 2>&1 || echo "pmc set $i failed" >> $OUT/bench.txt
done
