#!/bin/bash
# PMC counter passes (separate --pmc runs, kernel-trace only) over the bench-shape GEMMs of
# scripts/gemm_shapes.py. usage: gpu_shape_pmc.sh OUTDIR SHAPE:KIND:VARIANT_ENV ...
#   e.g. Wo:wgrad:DNA_WGRAD_IMPL=hip   Wo:fwd:-
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for job in "$@"; do
  IFS=: read shape kind envs <<< "$job"
  tag=${shape}_${kind}_$(echo "$envs" | tr -c 'A-Za-z0-9\n' '_')
  var="v"
  [ "$envs" != "-" ] && var="v,$envs"
  i=0
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_MFMA" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set -d $OUT/${tag}_$i -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/gemm_shapes.py --only $shape --kinds $kind --variants "$var" --rounds 1 --iters 2 > $OUT/${tag}_$i.log 2>&1 || echo "pmc set $i failed for $job" >> $OUT/errors.txt
  done
done
python $GRAFT_REPO_ROOT/scripts/pmc_table.py $OUT --kernel "gemm|wgrad|Cijk" > $OUT/summary.txt 2>&1 || true
cat $OUT/summary.txt
