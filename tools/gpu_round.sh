#!/bin/bash
# One GPU session: parity tests, bench, rocprof kernel stats. Each GPU step has its own limit.
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -3 gpurun_out/$TAG/pytest.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
timeout -k 10 300 python -u bench.py ${BENCH_ARGS} > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo "bench failed"; tail -30 gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --latency-batches 0 --serve-threads 0 --no-reload --configs-requests 0 ${BENCH_ARGS}) > gpurun_out/$TAG/rocprof.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/$TAG/rocprof.log; exit 1; }
find gpurun_out/$TAG/prof -name "*stats*"
