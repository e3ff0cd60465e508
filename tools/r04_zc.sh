#!/bin/bash
# Zero-copy small batches: GPU parity suite, then submit->results phases at 2,048 / 256 / 64 requests.
set -o pipefail
mkdir -p gpurun_out/zc
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/zc/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/zc/pytest.log; exit 1; }
tail -1 gpurun_out/zc/pytest.log
for n in 2048 256 64; do timeout -k 10 150 python -u tools/lat_phases.py $n 300 || exit 1; done
