#!/bin/bash
# Round 4: GPU parity suite, a C3 bench A/B against round 3's library (abx/libcedargpu_r03.so),
# then the full default bench line. Usage: tools/r04_check.sh TAG [extra ab settings...]
set -o pipefail
TAG=${1:-r04}; shift
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
bash tools/ab_multi.sh ${TAG}ab "CEDARGPU_AB_LIB=abx/libcedargpu_r03.so" "X=1" "$@" || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo "bench failed"; tail -20 gpurun_out/$TAG/bench.err; exit 1; }
python3 tools/bench_brief.py gpurun_out/$TAG/bench.json
