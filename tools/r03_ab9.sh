#!/bin/bash
set -o pipefail
TAG=${1:-r03ab9}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
CEDARGPU_SCAN_FILT=1 timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/$TAG/pytest_filt.log 2>&1 || { echo "pytest (filt) failed"; tail -30 gpurun_out/$TAG/pytest_filt.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest_filt.log
bash tools/ab_multi.sh $TAG "CEDARGPU_SCAN_FILT=1" "CEDARGPU_SCAN_FILT=0" || exit 1
CEDARGPU_SCAN_FILT=1 CEDARGPU_SCAN_STATS=1 timeout -k 10 240 python -u tools/c3_probe.py > gpurun_out/$TAG/scan_stats.log 2>&1 || { echo "scan stats failed"; tail -20 gpurun_out/$TAG/scan_stats.log; exit 1; }
grep -m 1 "scan stats" gpurun_out/$TAG/scan_stats.log || true
