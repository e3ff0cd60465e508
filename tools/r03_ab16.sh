#!/bin/bash
# Context lookups from (fingerprint, row) pairs; grouping key bits A/B.
set -o pipefail
TAG=${1:-r03ab16}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c5.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
bash tools/ab_multi.sh $TAG "CEDARGPU_GROUP_BITS=24" "CEDARGPU_GROUP_BITS=16" "CEDARGPU_GROUP_BITS=20" "CEDARGPU_GROUP_BITS=24" || exit 1
