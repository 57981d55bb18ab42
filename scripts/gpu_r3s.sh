#!/bin/bash
# Attention backward counters after the dS^T swizzle fix (bank-conflict share), plus the FFT
# passes' wait breakdown; one PMC set per rocprofv3 run.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3s
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d $O/attn_$i -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/attn_bench.py --b 512 --iters 3 --which bwd --dbias 1 > $O/attn_$i.log 2>&1 || { echo "pmc set $i failed"; tail -5 $O/attn_$i.log; exit 1; }
done
cd $GRAFT_REPO_ROOT && python scripts/pmc_table.py gpurun_out/r3s --kernel "bwd3_bf16_kernel" > gpurun_out/r3s/pmc_attn_bwd.txt 2>&1; cat gpurun_out/r3s/pmc_attn_bwd.txt
