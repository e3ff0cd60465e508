#!/bin/bash
# Device timeline (kernels + copies) of the 2,048-request submit->results loop.
set -o pipefail
mkdir -p gpurun_out/lat3
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/lat3/prof -o run -- python3 tools/lat_phases.py 2048 100 child > gpurun_out/lat3/prof.log 2>&1 || { tail -20 gpurun_out/lat3/prof.log; exit 1; }
find gpurun_out/lat3/prof -name '*.csv' | sort
