#!/bin/bash
# Bitonic index by bit ops, scan pair index by multiply: parity, bench, large-stage counters.
set -o pipefail
TAG=${1:-r03ab13}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
bash tools/ab_multi.sh $TAG "CEDARGPU_SCAN_FILT=1" "CEDARGPU_SCAN_FILT=1" || exit 1
CEDARGPU_BIG_STATS=1 timeout -k 10 240 python -u tools/c3_probe.py > gpurun_out/$TAG/big_stats.log 2>&1 || { echo "big stats failed"; tail -20 gpurun_out/$TAG/big_stats.log; exit 1; }
grep -m 2 -A1 "large stage stats" gpurun_out/$TAG/big_stats.log | tail -2 || true
