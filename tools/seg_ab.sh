#!/bin/bash
# Bench A/B over probe segment widths (and occupancy targets) on the default C3 workload.
# usage: tools/seg_ab.sh TAG "16 32 64" [extra bench args]
set -o pipefail
TAG=${1:-segab}
SEGS=${2:-"16 32 64"}
shift 2
mkdir -p gpurun_out/$TAG
for SEG in $SEGS; do
  CEDARGPU_PROBE_SEG=$SEG timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-batches 0 --serve-threads 0 --configs-requests 0 --no-reload --parity-sample 1024 "$@" > gpurun_out/$TAG/bench_$SEG.json 2> gpurun_out/$TAG/bench_$SEG.err || { echo "bench $SEG failed"; tail -20 gpurun_out/$TAG/bench_$SEG.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_$SEG.json')); c=d['config']; print('SEG $SEG', round(d['value']/1e6,1), 'M/s kernel_ms', round(d['roofline']['kernel_ms'],4), 'fu', c['device_followup_requests'], 'reruns', c['rerun_requests'], 'mism', d['parity_sample']['mismatches'])"
done
