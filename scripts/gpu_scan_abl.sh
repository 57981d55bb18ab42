#!/bin/bash
# A/B the selective-scan backward against ablation builds (dna_amd/lib/abl/lib<mask>.so)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in base "$@"; do
  if [ $m = base ]; then unset DNA_AMD_LIB; else export DNA_AMD_LIB=$GRAFT_REPO_ROOT/dna_amd/lib/abl/lib$m.so; fi
  echo -n "$m: " >> gpurun_out/scan_abl.txt
  timeout -k 10 120 python scripts/scan_bench.py --iters 3 2>/dev/null | grep "selective" >> gpurun_out/scan_abl.txt || exit 1
done
cat gpurun_out/scan_abl.txt
