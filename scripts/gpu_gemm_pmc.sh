#!/bin/bash
# PMC counter passes (separate --pmc runs, kernel-trace only) over single GEMM launches.
# usage: gpu_gemm_pmc.sh NAME:TAG [NAME:TAG ...]
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/gemm_pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for job in "$@"; do
  tag=${job/:/_}
  i=0
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SALU" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -k 10 180 rocprofv3 --kernel-trace --pmc $set -d $OUT/${tag}_$i -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/gemm_bench.py --only $job --iters 3 > $OUT/${tag}_$i.log 2>&1 || echo "pmc set $i failed for $job" >> $OUT/errors.txt
  done
done
python $GRAFT_REPO_ROOT/scripts/pmc_table.py $OUT > $OUT/summary.txt 2>&1 || true
