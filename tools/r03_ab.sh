#!/bin/bash
# Bench A/B of the round-3 changes (one bench per setting, C3 only), then a rocprof kernel split.
set -o pipefail
TAG=${1:-r03ab}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
bash tools/ab_multi.sh $TAG "CEDARGPU_SCAN_FILT=1" "CEDARGPU_SCAN_FILT=0" "CEDARGPU_GROUP_DEV=0" "CEDARGPU_GROUP=0" "CEDARGPU_BTAB_SLACK=8" || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --no-cpu-baseline --latency-batches 0 --serve-threads 0 --no-reload --configs-requests 0 --parity-sample 0) > gpurun_out/$TAG/rocprof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/$TAG/rocprof.log; exit 1; }
find gpurun_out/$TAG/prof -name "*kernel_stats*" -exec head -12 {} \;
