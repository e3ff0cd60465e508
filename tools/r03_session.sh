#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03a
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03a/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03a/pytest.log; exit 1; }
tail -2 gpurun_out/r03a/pytest.log
bash tools/ab_multi.sh r03a "CEDARGPU_SCAN_FILT=0" "CEDARGPU_SCAN_FILT=1" "CEDARGPU_SCAN_FILT=1 CEDARGPU_BTAB_SLACK=8"
