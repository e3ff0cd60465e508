#!/bin/bash
# rocprofv3 PMC passes over the timed launches (one counter group per pass, each under its own
# limit): where the probe kernel's wave cycles go (waiting vs issuing, by instruction class; counts
# are quad-cycles per the MI355X guide), then its instruction mix per wave.
set -o pipefail
TAG=${1:-stall}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --latency-batches 0 --parity-sample 0 --no-reload --serve-threads 0 --configs-requests 0 ${BENCH_ARGS}"
for PASS in "sq2 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
            "ins SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_BUSY_CYCLES"; do
  set -- $PASS
  P=$1
  shift
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$P -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS) > $OUT/$P.log 2>&1 || { echo "pass $P failed"; tail -20 $OUT/$P.log; exit 1; }
  python3 - "$OUT/$P" <<'PY'
import csv, glob, sys, collections
rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows = [r for r in rows if "cedar_probe_kernel<" in r["Kernel_Name"] and "1024u" not in r["Kernel_Name"]]
g = max(int(r["Grid_Size"]) for r in rows)
acc = collections.defaultdict(float)
disp = set()
for r in rows:
    if int(r["Grid_Size"]) == g:
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
        disp.add(r["Dispatch_Id"])
n = max(1, len(disp))
print({k: round(v / n) for k, v in sorted(acc.items())})
if "SQ_WAVE_CYCLES" in acc:
    w = acc["SQ_WAVE_CYCLES"] / n
    print({k: round(v / n / w, 3) for k, v in sorted(acc.items())}, "(fraction of SQ_WAVE_CYCLES)")
if "SQ_WAVES" in acc:
    w = acc["SQ_WAVES"] / n
    print({k: round(v / n / w, 1) for k, v in sorted(acc.items())}, "(per wave)")
PY
done
