#!/bin/bash
# Closure filings A/B on C3: scan-kernel register target 8 / 6 waves, closure filings off; then a
# rocprof kernel-stats pass of the default.
set -o pipefail
TAG=${1:-abcl}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
bash tools/ab_env.sh $TAG CEDARGPU_SCAN_OCC "8 6" || exit 1
bash tools/ab_env.sh $TAG/off CEDARGPU_NO_CLOSURE "1" || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --latency-batches 0 --serve-threads 0 --no-reload --configs-requests 0 --parity-sample 256) > gpurun_out/$TAG/rocprof.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/$TAG/rocprof.log; exit 1; }
head -5 gpurun_out/$TAG/prof/run_kernel_stats.csv
