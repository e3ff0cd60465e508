#!/bin/bash
# Round 4 profile of the C3 step at HEAD: scan / candidate-pass work counters, rocprofv3 kernel
# trace + stats of a short bench, then the per-kernel PMC passes (tools/pmc_kernels.sh).
set -o pipefail
TAG=${1:-r04prof}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
CEDARGPU_SCAN_STATS=1 CEDARGPU_CAND_STATS=1 timeout -k 10 240 python -u tools/c3_probe.py > gpurun_out/$TAG/stats.log 2>&1 || { echo "stats failed"; tail -20 gpurun_out/$TAG/stats.log; exit 1; }
grep -m 4 -A1 "stats:" gpurun_out/$TAG/stats.log || true
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/rocprof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --latency-batches 0 --serve-threads 0 --configs-requests 0 --no-reload --parity-sample 0 --no-submit-to-results) > gpurun_out/$TAG/rocprof_bench.json 2> gpurun_out/$TAG/rocprof.err || { echo "rocprof failed"; tail -20 gpurun_out/$TAG/rocprof.err; exit 1; }
find gpurun_out/$TAG/rocprof -name "*kernel_stats.csv" -exec head -12 {} \;
bash tools/pmc_kernels.sh $TAG/pmc
