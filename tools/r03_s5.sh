#!/bin/bash
# Session 5 at HEAD: the spill / counting-merge A/B against the previous commit's library
# (abx/libcedargpu_450c896.so), then the final round (GPU suite, smoke, bench, rocprof, PMC).
set -o pipefail
TAG=${1:-r03s5}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
bash tools/ab_multi.sh ${TAG}ab "CEDARGPU_AB_LIB=abx/libcedargpu_450c896.so" "CEDARGPU_CNT_RANK=0" "CEDARGPU_CNT_RANK=32" "CEDARGPU_AB_LIB=abx/libcedargpu_450c896.so" "CEDARGPU_CNT_RANK=32" || exit 1
bash tools/r03_final.sh $TAG || exit 1
