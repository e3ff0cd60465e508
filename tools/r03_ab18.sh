#!/bin/bash
# Candidate-pass occupancy A/B (4 waves per SIMD with spills vs 3 without).
set -o pipefail
TAG=${1:-r03ab18}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
bash tools/ab_multi.sh $TAG "CEDARGPU_CAND_OCC=4" "CEDARGPU_CAND_OCC=3" "CEDARGPU_CAND_OCC=4" "CEDARGPU_CAND_OCC=3" || exit 1
