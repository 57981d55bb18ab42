# PMC counter passes (separate rocprofv3 runs, kernel-trace only) over the attention backward
# micro-bench, with and without the fused bias-gradient sums. Results: gpurun_out/attn_bwd/
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/attn_bwd
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  for db in 1 0; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d $OUT/db${db}_$i -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/attn_bench.py --b 256 --iters 3 --which bwd --dbias $db > $OUT/db${db}_$i.log 2>&1
  done
done
