#!/bin/bash
# Same-session A/B of the round-3 scan / grouping changes against the round-2 final library.
set -o pipefail
TAG=${1:-r03ab5}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
bash tools/ab_multi.sh $TAG "CEDARGPU_AB_LIB=$PWD/ab/libcedargpu_r2.so" "CEDARGPU_SCAN_FILT=1" "CEDARGPU_SCAN_FILT=0" "CEDARGPU_GROUP_DEV=0" "CEDARGPU_GROUP_DEV=0 CEDARGPU_SCAN_FILT=0" "CEDARGPU_AB_LIB=$PWD/ab/libcedargpu_r2.so" || exit 1
