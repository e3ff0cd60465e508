#!/bin/bash
# Large stage SLIM form (bitmap merge, no hm words: 4 waves per SIMD) against the hm form; the
# candidate pass at 3 waves per SIMD rides along. GPU suite first (the SLIM form is the default).
set -o pipefail
TAG=${1:-r03ab19}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
for V in 0 3 4; do
  CEDARGPU_BIG_SLIM=$V CEDARGPU_BIG_STATS=1 timeout -k 10 240 python -u tools/c3_probe.py > gpurun_out/$TAG/big_stats_$V.log 2>&1 || { echo "big stats $V failed"; tail -20 gpurun_out/$TAG/big_stats_$V.log; exit 1; }
  echo "[CEDARGPU_BIG_SLIM=$V]"; grep -m 1 -A1 "large stage stats" gpurun_out/$TAG/big_stats_$V.log || true
done
bash tools/ab_multi.sh $TAG "CEDARGPU_BIG_SLIM=0" "CEDARGPU_BIG_SLIM=4" "CEDARGPU_BIG_SLIM=3" "CEDARGPU_BIG_SLIM=0" "CEDARGPU_BIG_SLIM=4" "CEDARGPU_CAND_OCC=3" || exit 1
