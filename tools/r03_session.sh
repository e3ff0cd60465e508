#!/bin/bash
# Round-3 session: GPU parity tests, then bench A/B of the scan's key-filter pass and the device
# grouping (each step under its own limit).
set -o pipefail
TAG=${1:-r03a}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
bash tools/ab_multi.sh $TAG "CEDARGPU_SCAN_FILT=1" "CEDARGPU_SCAN_FILT=0" "CEDARGPU_GROUP_DEV=0" "CEDARGPU_GROUP=0" "CEDARGPU_BTAB_SLACK=8"
