#!/bin/bash
# config-D FFT long-conv micro-benchmark for library variants (scripts/build_variant.sh):
#   bash scripts/fft_ab.sh "main base" [REPS]
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
for rep in $(seq ${2:-1}); do
  for l in $1; do
    if [ "$l" = main ]; then f=$ROOT/dna_amd/lib/libdna_amd.so; else f=$ROOT/dna_amd/lib/libdna_amd_$l.so; fi
    echo "$l: $(DNA_AMD_LIB=$f timeout -k 10 120 python $ROOT/scripts/fftconv_bench.py --B 2 --D 256 --L 65536 --dtype bf16 --bidirectional 1 --iters 10 2>/dev/null)"
  done
done
