#!/bin/bash
# Round 4: small-batch probe, host encode scaling with phase trace, then the C3 profile
# (tools/r04_prof.sh: work counters, rocprofv3 kernel stats, per-kernel PMC passes).
# Usage: tools/r04_prof2.sh TAG
set -o pipefail
TAG=${1:-r04p2}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
SIZES=64,256,1024,2048,4096 timeout -k 10 300 python -u tools/small_probe.py > gpurun_out/$TAG/small.log 2>&1 || { echo small failed; tail gpurun_out/$TAG/small.log; exit 1; }
cat gpurun_out/$TAG/small.log
CEDARGPU_TRACE_LAT=1 timeout -k 10 300 python tools/encode_scaling.py > gpurun_out/$TAG/enc.log 2>&1 || { echo enc failed; tail gpurun_out/$TAG/enc.log; exit 1; }
grep -v "^LAT" gpurun_out/$TAG/enc.log; grep "^LAT bulk" gpurun_out/$TAG/enc.log | tail -8
bash tools/r04_prof.sh $TAG/prof
