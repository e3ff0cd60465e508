#!/bin/bash
# Full GPU suite at the new defaults (bitset pass on), the enumerating scan's parity suite, bench A/B, scan stats.
set -o pipefail
TAG=${1:-r03ab11}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
CEDARGPU_SCAN_FILT=0 timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/$TAG/pytest_nofilt.log 2>&1 || { echo "pytest (no filt) failed"; tail -30 gpurun_out/$TAG/pytest_nofilt.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest_nofilt.log
bash tools/ab_multi.sh $TAG "CEDARGPU_SCAN_FILT=1" "CEDARGPU_SCAN_FILT=0" "CEDARGPU_GROUP_BITS=24" || exit 1
CEDARGPU_SCAN_STATS=1 timeout -k 10 240 python -u tools/c3_probe.py > gpurun_out/$TAG/scan_stats.log 2>&1 || { echo "scan stats failed"; tail -20 gpurun_out/$TAG/scan_stats.log; exit 1; }
grep -m 1 "scan stats" gpurun_out/$TAG/scan_stats.log || true
