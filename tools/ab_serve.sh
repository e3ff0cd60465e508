#!/bin/bash
# Serving-queue A/B: the bench's serving check (128 caller threads) per environment setting.
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
i=0
for SET in "$@"; do
  i=$((i+1))
  env $SET timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --latency-batches 2000 --configs-requests 0 --no-reload --parity-sample 256 > gpurun_out/$TAG/bench_$i.json 2> gpurun_out/$TAG/bench_$i.err || { echo "bench [$SET] failed"; tail -20 gpurun_out/$TAG/bench_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_$i.json')); s=d['serving']; l=d['latency']; print('[$SET] serving', round(s['decisions_per_s']), 'p50', s['p50_us'], 'p99', s['p99_us'], 'busy', round(s['device_busy_frac'],2), 'mean_batch', round(s['mean_batch'],1), '| batch lat p50/p99', round(l['p50_ms'],3), round(l['p99_ms'],3))"
done
