#!/bin/bash
# Counters of the Hyena short-conv kernels (one PMC set per rocprofv3 run) at config-D scale.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CMD="python $GRAFT_REPO_ROOT/scripts/hyena_op_bench.py --iters 3 --B 2"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d $O/p$i -o run --output-format csv -- $CMD > $O/p$i.log 2>&1 || { echo "set $i failed"; tail -5 $O/p$i.log; exit 1; }
done
cd $GRAFT_REPO_ROOT
for k in "shortconv_bwd_kernel" "shortconv_fwd_kernel" "gate_out_bwd" "gate_out_fwd"; do
  echo "== $k"; python scripts/pmc_table.py gpurun_out/r4b --kernel "$k" 2>&1 | grep -vE "^==" 
done
