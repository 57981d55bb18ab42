#!/bin/bash
# FFT conv after the row-pass LDS padding change: parity, bench, row/col PMC (conflicts).
set -o pipefail
O=gpurun_out/r3p
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_hyena.py tests/test_gpu_hyena_lm.py -q -x --timeout 300 --timeout-method thread > $O/fft_tests.log 2>&1 || { tail -30 $O/fft_tests.log; exit 1; }
tail -2 $O/fft_tests.log
for v in a b; do
  timeout -k 10 200 python scripts/fftconv_bench.py --dtype bf16,fp32 > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "== $v"; grep B= $O/bench_$v.log
done
cd /tmp && export TMPDIR=/tmp
CMD="python $GRAFT_REPO_ROOT/scripts/fftconv_bench.py --dtype fp32 --iters 3"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d $GRAFT_REPO_ROOT/$O/pmc -o run --output-format csv -- $CMD > $GRAFT_REPO_ROOT/$O/pmc.log 2>&1
cd $GRAFT_REPO_ROOT
for k in "col_fwd_kernel<float, 17>" "row_kernel<1, 17>" "col_inv_kernel<float, 0, 17>"; do
  echo "== $k"; python scripts/pmc_table.py $O --kernel "$k" 2>&1 | grep -E "share|IDX|CONFLICT" 
done
