#!/bin/bash
# Round 4: GPU parity suite, then the full default bench line (summary via tools/bench_brief.py).
set -o pipefail
TAG=${1:-r04full}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
CEDARGPU_TRACE_LAT=1 timeout -k 10 600 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo "bench failed"; tail -20 gpurun_out/$TAG/bench.err; exit 1; }
python3 tools/bench_brief.py gpurun_out/$TAG/bench.json
grep -m 6 "LAT bulk\|LAT split" gpurun_out/$TAG/bench.err || true
