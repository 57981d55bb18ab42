# attention micro-bench + PMC counter passes (separate --pmc runs, kernel-trace only)
# WHICH=fwd|bwd selects the pass; results: gpurun_out/attn/pmc*/ -> scripts/pmc_table.py
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/attn
WHICH=${WHICH:-fwd,bwd}
mkdir -p $OUT
timeout -k 10 120 python $GRAFT_REPO_ROOT/scripts/attn_bench.py --b 256 --which $WHICH > $OUT/bench.txt 2>&1
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d $OUT/pmc$i -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/attn_bench.py --b 256 --iters 3 --which $WHICH > $OUT/pmc$i.log 2>&1
done
