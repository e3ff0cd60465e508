#!/bin/bash
# Scan work profile (CEDARGPU_SCAN_STATS=1) on the C3 batch, bitset pass on and off.
set -o pipefail
TAG=${1:-r03st}
mkdir -p gpurun_out/$TAG
CEDARGPU_SCAN_FILT=1 CEDARGPU_SCAN_STATS=1 timeout -k 10 240 python -u tools/c3_probe.py > gpurun_out/$TAG/scan_stats_filt.log 2>&1 || { echo "scan stats failed"; tail -20 gpurun_out/$TAG/scan_stats_filt.log; exit 1; }
grep -m 1 "scan stats" gpurun_out/$TAG/scan_stats_filt.log || true
