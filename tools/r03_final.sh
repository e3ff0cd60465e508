#!/bin/bash
# Round-3 final measurements at HEAD: GPU suite, smoke, bench, rocprof kernel stats, per-kernel PMC.
set -o pipefail
TAG=${1:-r03fin}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
bash tools/gpu_round.sh $TAG || exit 1
bash tools/pmc_kernels.sh $TAG/pmc > gpurun_out/$TAG/pmc.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/$TAG/pmc.log; exit 1; }
tail -1 gpurun_out/$TAG/pmc.log
