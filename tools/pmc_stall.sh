#!/bin/bash
# One rocprofv3 PMC pass over the timed launches: where the probe kernel's wave cycles go
# (waiting vs issuing, by instruction class). Counts are quad-cycles per the MI355X guide.
set -o pipefail
TAG=${1:-stall}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --latency-batches 0 --parity-sample 0 --no-reload --serve-threads 0 --configs-requests 0 ${BENCH_ARGS}"
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM --output-format csv -d $OUT/sq2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS) > $OUT/sq2.log 2>&1 || { echo "pass failed"; tail -20 $OUT/sq2.log; exit 1; }
python3 - "$OUT/sq2" <<'PY'
import csv, glob, sys, collections
rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows = [r for r in rows if "cedar_probe_kernel<16u, 64u, 4u, false" in r["Kernel_Name"]]
g = max(int(r["Grid_Size"]) for r in rows)
acc = collections.defaultdict(float)
disp = set()
for r in rows:
    if int(r["Grid_Size"]) == g:
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
        disp.add(r["Dispatch_Id"])
n = max(1, len(disp))
w = acc["SQ_WAVE_CYCLES"] / n
print({k: round(v / n) for k, v in sorted(acc.items())})
print({k: round(v / n / w, 3) for k, v in sorted(acc.items())}, "(fraction of SQ_WAVE_CYCLES)")
PY
