#!/bin/bash
# A whole source tree of another git revision (default HEAD) with its native library built, as
# _ab/<name>/ inside the repo (so it travels to the GPU box), for interleaved A/B runs of changes
# that touch the Python side and the C ABI together: scripts/gpu.sh ab-tree "main base" runs
# bench.py of the working tree and _ab/base/bench.py alternately.
set -e
REV=${1:-HEAD}
NAME=${2:-base}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
DST="$ROOT/_ab/$NAME"
rm -rf "$DST"
mkdir -p "$DST"
git -C "$ROOT" archive "$REV" | tar -x -C "$DST"
rm -rf "$DST/tests/golden" "$DST/profiles"
mkdir -p "$DST/build/native"
(cd "$DST" && python -m dna_amd.build > /dev/null)
rm -rf "$DST/build"
echo "built $DST from $REV"
