#!/bin/bash
# Bench A/B over several environment settings, one bench per setting (C3, no extras):
#   tools/ab_multi.sh TAG "A=1 B=2" "A=3" ... 
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
i=0
for SET in "$@"; do
  i=$((i+1))
  env $SET timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-batches 0 --serve-threads 0 --configs-requests 0 --no-reload --parity-sample 1024 > gpurun_out/$TAG/bench_$i.json 2> gpurun_out/$TAG/bench_$i.err || { echo "bench [$SET] failed"; tail -20 gpurun_out/$TAG/bench_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_$i.json')); c=d['config']; print('[$SET]', round(d['value']/1e6,1), 'M/s kernel_ms', round(d['roofline']['kernel_ms'],4), 'fu', c['device_followup_requests'], 'reruns', c['rerun_requests'], 'mism', d['parity_sample']['mismatches'], 'phases', {k: round(v,3) for k,v in d['roofline'].get('phases_ms',{}).items()})"
done
