# FFT long-conv micro-bench + PMC counter passes (separate --pmc runs, kernel-trace only)
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/fftpmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d $OUT/pmc$i -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/fftconv_bench.py --dtype fp32 --iters 2 > $OUT/pmc$i.log 2>&1
done
