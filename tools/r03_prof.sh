#!/bin/bash
# Candidate-pass work counters, then the per-kernel PMC passes (vL1D, instruction mix, LDS bank
# conflicts, HBM fetch / write) of the complete step at HEAD.
set -o pipefail
TAG=${1:-r03prof}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
CEDARGPU_CAND_STATS=1 timeout -k 10 240 python -u tools/c3_probe.py > gpurun_out/$TAG/cand_stats.log 2>&1 || { echo "cand stats failed"; tail -20 gpurun_out/$TAG/cand_stats.log; exit 1; }
grep -m 2 -A1 "candidate pass stats" gpurun_out/$TAG/cand_stats.log || true
bash tools/pmc_kernels.sh $TAG/pmc
