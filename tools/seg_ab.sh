#!/bin/bash
# GPU parity tests with the default probe segment width, then bench A/B over segment widths.
set -o pipefail
TAG=${1:-segab}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
for SEG in 16 32 64 16; do
  CEDARGPU_PROBE_SEG=$SEG timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-batches 50 --parity-sample 1024 > gpurun_out/$TAG/bench_$SEG.json 2> gpurun_out/$TAG/bench_$SEG.err || { echo "bench $SEG failed"; tail -20 gpurun_out/$TAG/bench_$SEG.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_$SEG.json')); print('SEG $SEG', round(d['value']/1e6,1), 'M/s kernel_ms', round(d['roofline']['kernel_ms'],4), 'p99', round(d['latency']['p99_ms'],3), 'mism', d['parity_sample']['mismatches'])"
done
