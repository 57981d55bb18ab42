#!/bin/bash
# Build the native library of another git revision (default HEAD, i.e. without the working
# tree's uncommitted edits) as dna_amd/lib/libdna_amd_<name>.so, for in-process A/B runs on the
# GPU box: DNA_AMD_LIB=dna_amd/lib/libdna_amd_<name>.so python bench.py ... (scripts/gpu.sh ab-lib).
set -e
REV=${1:-HEAD}
NAME=${2:-base}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d /tmp/dna_variant.XXXXXX)
git -C "$ROOT" archive "$REV" | tar -x -C "$TMP"
mkdir -p "$TMP/build/native"
# reuse object files of unchanged sources (same content => same object)
# (DNA_AMD_FILE_FLAGS in the environment adds per-file compiler flags: dna_amd/build.py)
(cd "$TMP" && python -m dna_amd.build > /dev/null)
cp "$TMP/dna_amd/lib/libdna_amd.so" "$ROOT/dna_amd/lib/libdna_amd_$NAME.so"
rm -rf "$TMP"
echo "built $ROOT/dna_amd/lib/libdna_amd_$NAME.so from $REV"
