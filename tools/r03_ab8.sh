#!/bin/bash
# The two-level scope-bitset scan: GPU parity under CEDARGPU_SCAN_FILT=1, then bench A/B and scan stats.
set -o pipefail
TAG=${1:-r03ab8}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
CEDARGPU_SCAN_FILT=1 timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c5.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/$TAG/pytest_filt.log 2>&1 || { echo "pytest (filt) failed"; tail -30 gpurun_out/$TAG/pytest_filt.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest_filt.log
bash tools/ab_multi.sh $TAG "CEDARGPU_SCAN_FILT=1" "CEDARGPU_SCAN_FILT=0" "CEDARGPU_SCAN_FILT=1 CEDARGPU_GROUP_DEV=0" "CEDARGPU_SCAN_FILT=0 CEDARGPU_GROUP_DEV=0" || exit 1
CEDARGPU_SCAN_FILT=1 CEDARGPU_SCAN_STATS=1 timeout -k 10 240 python -u tools/c3_probe.py > gpurun_out/$TAG/scan_stats.log 2>&1 || { echo "scan stats failed"; tail -20 gpurun_out/$TAG/scan_stats.log; exit 1; }
grep -m 2 "scan stats" gpurun_out/$TAG/scan_stats.log || true
