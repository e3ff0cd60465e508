#!/bin/bash
set -o pipefail
TAG=${1:-r03ab2}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
bash tools/ab_multi.sh $TAG "CEDARGPU_SCAN_FILT=0" "CEDARGPU_SCAN_FILT=0 CEDARGPU_GROUP_DEV=0" "CEDARGPU_SCAN_FILT=1" || exit 1
CEDARGPU_SCAN_FILT=0 bash tools/pmc_kernels.sh $TAG/pmc
