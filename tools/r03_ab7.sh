#!/bin/bash
# GPU parity suite, then bench A/B: device radix grouping (32 / 24 key bits) vs the host sort vs none.
set -o pipefail
TAG=${1:-r03ab7}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
bash tools/ab_multi.sh $TAG "CEDARGPU_GROUP_BITS=32" "CEDARGPU_GROUP_BITS=24" "CEDARGPU_GROUP_DEV=0" "CEDARGPU_GROUP=0" || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --no-cpu-baseline --latency-batches 0 --serve-threads 0 --no-reload --configs-requests 0 --parity-sample 0) > gpurun_out/$TAG/rocprof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/$TAG/rocprof.log; exit 1; }
