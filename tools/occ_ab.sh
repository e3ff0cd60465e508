#!/bin/bash
# Bench A/B over the probe kernel's register-allocation occupancy target (16-lane segments).
set -o pipefail
TAG=${1:-occab}
mkdir -p gpurun_out/$TAG
for OCC in 1 4 5 1 4 5; do
  CEDARGPU_PROBE_OCC=$OCC timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-batches 20 --parity-sample 1024 > gpurun_out/$TAG/bench_$OCC.json 2> gpurun_out/$TAG/bench_$OCC.err || { echo "bench $OCC failed"; tail -20 gpurun_out/$TAG/bench_$OCC.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_$OCC.json')); print('OCC $OCC', round(d['value']/1e6,1), 'M/s kernel_ms', round(d['roofline']['kernel_ms'],4), 'mism', d['parity_sample']['mismatches'])"
done
