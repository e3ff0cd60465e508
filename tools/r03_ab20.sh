#!/bin/bash
# Candidate-pass merge: ranks by counting for small merges (CEDARGPU_CNT_RANK, default 32) against
# the bitonic network (0), and the merge's recomputed indices (candidate-pass spills 36 -> 8 B per
# lane) against the previous commit's library (ab/libcedargpu_450c896.so). GPU suite first.
set -o pipefail
TAG=${1:-r03ab20}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
for V in 0 32; do
  CEDARGPU_CNT_RANK=$V CEDARGPU_CAND_STATS=1 timeout -k 10 240 python -u tools/c3_probe.py > gpurun_out/$TAG/cand_stats_$V.log 2>&1 || { echo "cand stats $V failed"; tail -20 gpurun_out/$TAG/cand_stats_$V.log; exit 1; }
  echo "[CEDARGPU_CNT_RANK=$V]"; grep -m 1 -A1 "candidate pass stats" gpurun_out/$TAG/cand_stats_$V.log || true
done
bash tools/ab_multi.sh $TAG "CEDARGPU_AB_LIB=ab/libcedargpu_450c896.so" "CEDARGPU_CNT_RANK=0" "CEDARGPU_CNT_RANK=32" "CEDARGPU_CNT_RANK=64" "CEDARGPU_AB_LIB=ab/libcedargpu_450c896.so" "CEDARGPU_CNT_RANK=0" "CEDARGPU_CNT_RANK=32" || exit 1
