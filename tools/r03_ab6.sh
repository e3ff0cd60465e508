#!/bin/bash
# GPU parity suite, then bench A/B: device bucket grouping (20 / 22 bits) vs the host sort, scan bitsets.
set -o pipefail
TAG=${1:-r03ab6}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
bash tools/ab_multi.sh $TAG "CEDARGPU_GROUP_BITS=20" "CEDARGPU_GROUP_BITS=22" "CEDARGPU_GROUP_DEV=0" "CEDARGPU_SCAN_FILT=1" "CEDARGPU_GROUP_BITS=16" || exit 1
CEDARGPU_SCAN_STATS=1 timeout -k 10 240 python -u tools/c3_probe.py > gpurun_out/$TAG/scan_stats.log 2>&1 || { echo "scan stats failed"; tail -20 gpurun_out/$TAG/scan_stats.log; exit 1; }
grep -m 3 "scan stats" gpurun_out/$TAG/scan_stats.log || true
