#!/bin/bash
# Small-batch latency: phases with glibc's heap trimming off, then a device timeline of the 2,048-request loop.
set -o pipefail
mkdir -p gpurun_out/lat2
export TMPDIR=/tmp
MALLOC_TRIM_THRESHOLD_=1073741824 MALLOC_MMAP_THRESHOLD_=1073741824 MALLOC_TOP_PAD_=67108864 timeout -k 10 150 python -u tools/lat_phases.py 2048 300 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/lat2/prof -o run -- python3 tools/lat_phases.py 2048 200 child > gpurun_out/lat2/prof.log 2>&1 || { tail -20 gpurun_out/lat2/prof.log; exit 1; }
find gpurun_out/lat2/prof -name '*.csv' | sort
