#!/bin/bash
# A/B of the 8-lane probe kernel's register target (3 waves per SIMD unconstrained vs 4 forced).
set -o pipefail
mkdir -p gpurun_out/ab_occ8
for O in 3 4; do
  CEDARGPU_PROBE_OCC=$O timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-batches 0 --serve-threads 0 --configs-requests 0 --no-reload --parity-sample 1024 --steps 5 > gpurun_out/ab_occ8/occ_$O.json 2> gpurun_out/ab_occ8/occ_$O.err || { echo "occ $O failed"; tail -5 gpurun_out/ab_occ8/occ_$O.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_occ8/occ_$O.json')); print('OCC $O', round(d['value']/1e6,1), 'M/s ms', round(d['roofline']['kernel_ms'],3), 'mism', d['parity_sample']['mismatches'])"
done
