#!/bin/bash
# Same-session bisect of the round-3 scan slowdown: each commit's library under the host grouping
# with the scan's filter pass off (the round-2 kernel path where the knobs exist).
set -o pipefail
TAG=${1:-r03bis}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
K="CEDARGPU_GROUP_DEV=0 CEDARGPU_SCAN_FILT=0"
bash tools/ab_multi.sh $TAG "CEDARGPU_AB_LIB=$PWD/ab/libcedargpu_r2.so" "$K CEDARGPU_AB_LIB=$PWD/ab/libcedargpu_4729cf1.so" "$K CEDARGPU_AB_LIB=$PWD/ab/libcedargpu_c9019e7.so" "$K CEDARGPU_AB_LIB=$PWD/ab/libcedargpu_5ef4ed1.so" "$K CEDARGPU_AB_LIB=$PWD/ab/libcedargpu_2796b0a.so" "$K CEDARGPU_AB_LIB=$PWD/ab/libcedargpu_ca0c479.so" "$K" || exit 1
