#!/bin/bash
# Bench A/B over one environment variable: tools/ab_env.sh TAG VAR "v1 v2 ..." [bench args]
set -o pipefail
TAG=$1; VAR=$2; VALS=$3
shift 3
mkdir -p gpurun_out/$TAG
for V in $VALS; do
  env $VAR=$V timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-batches 0 --serve-threads 0 --configs-requests 0 --no-reload --parity-sample 1024 "$@" > gpurun_out/$TAG/bench_$V.json 2> gpurun_out/$TAG/bench_$V.err || { echo "bench $V failed"; tail -20 gpurun_out/$TAG/bench_$V.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_$V.json')); c=d['config']; print('$VAR=$V', round(d['value']/1e6,1), 'M/s kernel_ms', round(d['roofline']['kernel_ms'],4), 'fu', c['device_followup_requests'], 'reruns', c['rerun_requests'], 'mism', d['parity_sample']['mismatches'])"
done
