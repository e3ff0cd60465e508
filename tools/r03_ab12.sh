#!/bin/bash
# Heavy requests past the candidate pass (+ its early stop on overflow): GPU parity, then A/B.
set -o pipefail
TAG=${1:-r03ab12}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c5.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
bash tools/ab_multi.sh $TAG "CEDARGPU_SCAN_HEAVY=128" "CEDARGPU_SCAN_HEAVY=1000000" "CEDARGPU_SCAN_HEAVY=64" "CEDARGPU_SCAN_HEAVY=96" || exit 1
CEDARGPU_CAND_STATS=1 timeout -k 10 240 python -u tools/c3_probe.py > gpurun_out/$TAG/cand_stats.log 2>&1 || { echo "cand stats failed"; tail -20 gpurun_out/$TAG/cand_stats.log; exit 1; }
grep -m 1 -A1 "candidate pass stats" gpurun_out/$TAG/cand_stats.log || true
