#!/bin/bash
# like compares with batched byte loads: parity (like cases) + bench + candidate counters.
set -o pipefail
TAG=${1:-r03ab17}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_admission.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
bash tools/ab_multi.sh $TAG "CEDARGPU_SCAN_FILT=1" "CEDARGPU_SCAN_FILT=1" || exit 1
