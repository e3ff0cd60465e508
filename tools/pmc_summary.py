"""Reduces rocprofv3 --pmc CSV passes (tools/pmc.sh) to per-launch averages for the full-size
dispatches of the evaluation kernel. HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reads half the bytes of wide (16 B/lane) reads, so the
read side is doubled (the kernel's global reads are 16-byte vector loads of heads / index slots
and dword gathers; the doubling is the guide's calibration for the wide ones)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNEL = os.environ.get("PMC_KERNEL", "cedar_probe_kernel")  # substring of the kernel name


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def main(out):
    per = defaultdict(lambda: defaultdict(list))  # counter -> dispatch -> values
    grids = {}
    for sub in sorted(os.listdir(out)):
        d = os.path.join(out, sub)
        if not os.path.isdir(d):
            continue
        for r in load(d):
            if KERNEL not in r.get("Kernel_Name", ""):
                continue
            key = (sub, r.get("Dispatch_Id"))
            grids[key] = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
            per[r["Counter_Name"]][key].append(float(r["Counter_Value"]))
    if not grids:
        print(json.dumps({"error": "no dispatches of " + KERNEL}))
        return
    gmax = max(grids.values())
    res = {"kernel": KERNEL, "grid_size": gmax}
    for c, disp in per.items():
        vals = [sum(v) for k, v in disp.items() if grids[k] == gmax]
        if vals:
            res[c] = sum(vals) / len(vals)
    if "FETCH_SIZE" in res and "WRITE_SIZE" in res:
        res["hbm_read_bytes_per_launch"] = res["FETCH_SIZE"] * 1024 * 2
        res["hbm_write_bytes_per_launch"] = res["WRITE_SIZE"] * 1024
        res["hbm_bytes_per_launch"] = res["hbm_read_bytes_per_launch"] + res["hbm_write_bytes_per_launch"]
    if "TCC_HIT_sum" in res and "TCC_MISS_sum" in res:
        tot = res["TCC_HIT_sum"] + res["TCC_MISS_sum"]
        res["l2_hit_rate"] = res["TCC_HIT_sum"] / tot if tot else None
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
