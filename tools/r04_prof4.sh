#!/bin/bash
# Round 4 profiles without the bench line (already in gpurun_out/TAG): rocprofv3 kernel stats of a
# short bench, the per-kernel PMC passes, the host encode. Usage: tools/r04_prof4.sh TAG
set -o pipefail
TAG=${1:-r04final}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/rocprof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --latency-batches 0 --serve-threads 0 --configs-requests 0 --no-reload --parity-sample 0 --no-submit-to-results) > gpurun_out/$TAG/rocprof_bench.json 2> gpurun_out/$TAG/rocprof.err || { echo "rocprof failed"; tail -20 gpurun_out/$TAG/rocprof.err; exit 1; }
find gpurun_out/$TAG/rocprof -name "*kernel_stats.csv" -exec head -12 {} \;
bash tools/pmc_kernels.sh $TAG/pmc || exit 1
CEDARGPU_HOST_THREADS=16 timeout -k 10 120 python tools/encode_scaling.py child > gpurun_out/$TAG/enc.log 2>&1 && cat gpurun_out/$TAG/enc.log
CEDARGPU_COMPILE_TIMES=1 timeout -k 10 200 python tools/c5_compile.py > gpurun_out/$TAG/c5_compile.log 2>&1 && grep -A40 "=== incremental" gpurun_out/$TAG/c5_compile.log
