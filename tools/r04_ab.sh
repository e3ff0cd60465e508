#!/bin/bash
# A/B of the step: abx/libcedargpu_base.so (CEDARGPU_AB_LIB) against the in-tree build, two runs
# each, alternating. Usage: tools/r04_ab.sh TAG
set -o pipefail
TAG=${1:-ab}
mkdir -p gpurun_out/$TAG
ARGS="--steps 30 --warmup 3 --no-cpu-baseline --latency-batches 0 --serve-threads 0 --configs-requests 0 --no-reload --parity-sample 0 --no-submit-to-results"
for r in 1 2; do
  CEDARGPU_AB_LIB=$GRAFT_REPO_ROOT/abx/libcedargpu_base.so timeout -k 10 200 python bench.py $ARGS > gpurun_out/$TAG/base_$r.json 2> gpurun_out/$TAG/base_$r.err || { echo "base failed"; tail -5 gpurun_out/$TAG/base_$r.err; exit 1; }
  timeout -k 10 200 python bench.py $ARGS > gpurun_out/$TAG/new_$r.json 2> gpurun_out/$TAG/new_$r.err || { echo "new failed"; tail -5 gpurun_out/$TAG/new_$r.err; exit 1; }
done
for f in gpurun_out/$TAG/*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); r=d['roofline']
print('$f', '%.4g'%d['value'], {k: round(v,3) for k,v in r.get('phases_ms',{}).items()})"; done
