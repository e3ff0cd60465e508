#!/bin/bash
# GPU parity tests, the C3 probe-kernel work profile and a short bench (each step under its own limit).
set -o pipefail
TAG=${1:-quick}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
CEDARGPU_PROBE_STATS=1 timeout -k 10 240 python -u tools/c3_probe.py > gpurun_out/$TAG/c3_stats.log 2>&1 || { echo "c3 stats failed"; tail -20 gpurun_out/$TAG/c3_stats.log; exit 1; }
grep -A1 "requests 1048576" gpurun_out/$TAG/c3_stats.log | tail -2
timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-batches 2000 --serve-threads 0 --no-reload ${BENCH_ARGS} > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo "bench failed"; tail -20 gpurun_out/$TAG/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/$TAG/bench.json')); c=d['config']
print('C3', round(d['value']/1e6,1), 'M/s ms', round(d['ms_per_step'],3), 'frac', d['roofline']['frac'], 'fu', c['device_followup_requests'], 'reruns', c['rerun_requests'], 'parity', d['parity_sample'])
for k,v in d.get('configs',{}).items(): print(k, 'kernel_ms', round(v['kernel_ms'],4), 's2r', round(v['submit_to_results_ms'],3), 'parity', v['parity_sample']['mismatches'])
print('latency', d.get('latency',{}).get('p50_ms'), d.get('latency',{}).get('p99_ms'))
"
