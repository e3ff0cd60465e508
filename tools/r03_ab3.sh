#!/bin/bash
set -o pipefail
TAG=${1:-r03ab3}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
bash tools/ab_multi.sh $TAG "CEDARGPU_SCAN_FILT=1" "CEDARGPU_SCAN_FILT=0" "CEDARGPU_SCAN_FILT=1 CEDARGPU_BTAB_SLACK=8" "CEDARGPU_SCAN_FILT=1 CEDARGPU_GROUP_DEV=0" "CEDARGPU_GROUP_KEY=uid" || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --no-cpu-baseline --latency-batches 0 --serve-threads 0 --no-reload --configs-requests 0 --parity-sample 0) > gpurun_out/$TAG/rocprof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/$TAG/rocprof.log; exit 1; }
python3 -c "
import csv,glob
for f in glob.glob('gpurun_out/$TAG/prof/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)): print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg', r['Percentage'])
"
