#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_multi.sh r04fab "CEDARGPU_AB_LIB=abx/libcedargpu_r03.so" "X=1" "CEDARGPU_CLOSURE_CACHE=1" || exit 1
mkdir -p gpurun_out/r04f
timeout -k 10 600 python -u bench.py > gpurun_out/r04f/bench.json 2> gpurun_out/r04f/bench.err || { echo "bench failed"; tail -20 gpurun_out/r04f/bench.err; exit 1; }
python3 tools/bench_brief.py gpurun_out/r04f/bench.json
