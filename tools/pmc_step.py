"""Reduces rocprofv3 --pmc passes (tools/pmc_kernels.sh) to per-step figures of the complete C3
evaluation step: every dispatch from one full-size cedar_scan_kernel launch up to the next scan
launch (candidate pass, gather, follow-ups), summed, averaged over the timed steps. HBM bytes follow
MI355X_MICROARCH.md (FETCH_SIZE / WRITE_SIZE in KiB; the gfx950 read side doubled). Writes the
profiles/pmc_latest.json shape bench.py reads for `roofline.traffic`."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def dispatches(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    per = defaultdict(lambda: {"name": "", "grid": 0, "c": defaultdict(float)})
    for r in rows:
        k = int(r["Dispatch_Id"])
        per[k]["name"] = r["Kernel_Name"]
        per[k]["grid"] = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
        per[k]["c"][r["Counter_Name"]] += float(r["Counter_Value"])
    return [per[k] for k in sorted(per)]


def steps(ds):
    gmax = max((d["grid"] for d in ds if "cedar_scan_kernel" in d["name"]), default=0)
    out, cur = [], None
    for d in ds:
        if "cedar_scan_kernel" in d["name"]:
            if cur:
                out.append(cur)
            cur = [d] if d["grid"] == gmax else None
        elif cur is not None and "rocclr" not in d["name"]:
            cur.append(d)
    if cur:
        out.append(cur)
    return out


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def main(out, policies, batch, hierarchy):
    res = {"policies": policies, "batch": batch, "hierarchy": hierarchy, "kernels": {}}
    tot = defaultdict(float)
    for sub in ("fetch", "write", "tcp", "sq", "lds"):
        d = os.path.join(out, sub)
        if not os.path.isdir(d):
            continue
        st = steps(dispatches(d))
        if not st:
            continue
        for s in st:
            for x in s:
                for c, v in x["c"].items():
                    tot[c] += v / len(st)
                    kk = res["kernels"].setdefault(short(x["name"]) + f" grid {x['grid']}", {})
                    kk[c] = kk.get(c, 0.0) + v / len(st)
        res["steps_" + sub] = len(st)
    res.update(tot)
    if "FETCH_SIZE" in res and "WRITE_SIZE" in res:
        res["hbm_read_bytes_per_launch"] = res["FETCH_SIZE"] * 1024 * 2
        res["hbm_write_bytes_per_launch"] = res["WRITE_SIZE"] * 1024
        res["hbm_bytes_per_launch"] = res["hbm_read_bytes_per_launch"] + res["hbm_write_bytes_per_launch"]
        res["what"] = "one complete step (scan + candidate pass + gather + follow-ups), per 1M-request launch"
    for k in res["kernels"].values():  # share of LDS-active cycles lost to bank conflicts
        if k.get("SQ_LDS_IDX_ACTIVE"):
            k["lds_bank_conflict_frac"] = k.get("SQ_LDS_BANK_CONFLICT", 0.0) / k["SQ_LDS_IDX_ACTIVE"]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4])
