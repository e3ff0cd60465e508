#!/bin/bash
# Round 4 iteration run: GPU parity suite, C3 bench A/B against round 3's library, small-batch
# probe. Usage: tools/r04_run.sh TAG
set -o pipefail
TAG=${1:-r04}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
bash tools/ab_multi.sh ${TAG}ab "CEDARGPU_AB_LIB=abx/libcedargpu_r03.so" "X=1" || exit 1
SIZES=64,256,1024,2048,4096 timeout -k 10 300 python -u tools/small_probe.py > gpurun_out/$TAG/small.log 2>&1 || { echo small failed; tail gpurun_out/$TAG/small.log; exit 1; }
cat gpurun_out/$TAG/small.log
