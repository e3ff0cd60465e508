#!/bin/bash
# Round 4 measurement: GPU suite, the full default bench line, rocprofv3 kernel stats of a short
# bench, the per-kernel PMC passes (profiles/pmc_latest.json source), and the host encode with
# huge-page blocks (A/B). Usage: tools/r04_final.sh TAG
set -o pipefail
TAG=${1:-r04final}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
bash tools/r04_full.sh $TAG || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/rocprof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --latency-batches 0 --serve-threads 0 --configs-requests 0 --no-reload --parity-sample 0 --no-submit-to-results) > gpurun_out/$TAG/rocprof_bench.json 2> gpurun_out/$TAG/rocprof.err || { echo "rocprof failed"; tail -20 gpurun_out/$TAG/rocprof.err; exit 1; }
find gpurun_out/$TAG/rocprof -name "*kernel_stats.csv" -exec head -12 {} \;
bash tools/pmc_kernels.sh $TAG/pmc || exit 1
CEDARGPU_HUGEPAGES=1 CEDARGPU_HOST_THREADS=16 timeout -k 10 120 python tools/encode_scaling.py child > gpurun_out/$TAG/enc_huge.log 2>&1 && cat gpurun_out/$TAG/enc_huge.log
CEDARGPU_HOST_THREADS=16 timeout -k 10 120 python tools/encode_scaling.py child > gpurun_out/$TAG/enc.log 2>&1 && cat gpurun_out/$TAG/enc.log
