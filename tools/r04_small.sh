#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04h
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r04h/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r04h/pytest.log; exit 1; }
tail -1 gpurun_out/r04h/pytest.log
SIZES=16,64,256,1024,2048,4096 timeout -k 10 300 python -u tools/small_probe.py > gpurun_out/r04h/small.log 2>&1 || { echo small failed; tail gpurun_out/r04h/small.log; exit 1; }
cat gpurun_out/r04h/small.log
