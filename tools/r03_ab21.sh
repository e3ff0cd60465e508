#!/bin/bash
# Large stage SLIM form at 3 waves per SIMD (168 VGPRs, no spills) against 4 (128 VGPRs, 88 B per
# lane of spills), three benches each, interleaved.
set -o pipefail
TAG=${1:-r03ab21}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
bash tools/ab_multi.sh $TAG "CEDARGPU_BIG_SLIM=4" "CEDARGPU_BIG_SLIM=3" "CEDARGPU_BIG_SLIM=4" "CEDARGPU_BIG_SLIM=3" "CEDARGPU_BIG_SLIM=4" "CEDARGPU_BIG_SLIM=3" || exit 1
