#!/bin/bash
# Bench A/B over environment settings of the probe kernel: tools/ab_probe.sh TAG "NAME:VAR=V,VAR=V ..." [bench args]
set -o pipefail
TAG=$1; CASES=$2
shift 2
mkdir -p gpurun_out/$TAG
for C in $CASES; do
  N=${C%%:*}; E=${C#*:}
  env $(echo $E | tr ',' ' ') timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-batches 0 --serve-threads 0 --configs-requests 0 --no-reload --parity-sample 1024 --steps 5 "$@" > gpurun_out/$TAG/$N.json 2> gpurun_out/$TAG/$N.err || { echo "$N failed"; tail -5 gpurun_out/$TAG/$N.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/$TAG/$N.json')); print('$N', round(d['value']/1e6,1), 'M/s ms', round(d['roofline']['kernel_ms'],3), 'mism', d['parity_sample']['mismatches'])"
done
