#!/bin/bash
# The large stage's work counters on the C3 batch.
set -o pipefail
TAG=${1:-r03big}
mkdir -p gpurun_out/$TAG
CEDARGPU_BIG_STATS=1 timeout -k 10 240 python -u tools/c3_probe.py > gpurun_out/$TAG/big_stats.log 2>&1 || { echo "big stats failed"; tail -20 gpurun_out/$TAG/big_stats.log; exit 1; }
grep -m 2 -A1 "large stage stats" gpurun_out/$TAG/big_stats.log || true
