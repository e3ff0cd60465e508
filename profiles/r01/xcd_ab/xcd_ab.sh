#!/bin/bash
# A/B of request order x XCD-contiguous block mapping on the C3 bench (one GPU session).
set -o pipefail
OUT=gpurun_out/xcd_ab
mkdir -p $OUT
A="--no-cpu-baseline --latency-batches 0 --serve-threads 0 --no-reload --configs-requests 0 --parity-sample 256 ${BENCH_ARGS}"
for order in random user; do
  for remap in 0 1; do
    CEDARGPU_XCD_REMAP=$remap timeout -k 10 200 python -u bench.py $A --order $order > $OUT/${order}_$remap.json 2> $OUT/${order}_$remap.err || { echo "run $order $remap failed"; tail -5 $OUT/${order}_$remap.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/${order}_$remap.json')); print('$order', $remap, round(d['value']/1e6,1), 'M/s kernel_ms', round(d['roofline']['kernel_ms'],4), 'parity', d['parity_sample']['mismatches'])"
  done
done
