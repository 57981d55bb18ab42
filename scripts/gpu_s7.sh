#!/bin/bash
# Round measurement bundle at the new default per-GPU batch (512), then the HipLinear checks.
set -o pipefail
ROUND=r02b512 BATCH=512 timeout -k 10 800 bash scripts/gpu_round_profile.sh || exit 1
cd $GRAFT_REPO_ROOT && bash scripts/gpu_s6.sh
