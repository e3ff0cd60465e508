"""One-screen summary of a bench.py JSON line (GPU run logs)."""
import json
import sys

d = json.load(open(sys.argv[1]))
r = d["roofline"]
print("C3 %.3g dec/s  ms/step %.3f  dominant %s %.3f ms frac %.4f  step_frac %.4f" % (
    d["value"], d["ms_per_step"], r.get("dominant_phase"), r.get("dominant_kernel_ms", 0), r["frac"], r.get("step_frac", 0)))
print("phases", {k: round(v, 3) for k, v in r.get("phases_ms", {}).items()})
print("transfer", d.get("transfer"))
print("s2r_1m", {k: v for k, v in (d.get("submit_to_results_1m") or {}).items() if k != "what"})
print("host", d.get("host"), "parity", d.get("parity_sample"))
lat = d.get("latency") or {}
print("latency 2048: p50 %s p99 %s p999 %s" % (lat.get("p50_ms"), lat.get("p99_ms"), lat.get("p999_ms")))
sv = d.get("serving") or {}
print("serving best<1ms %s @%s threads; curve %s" % (sv.get("best_under_1ms"), sv.get("best_under_1ms_threads"),
                                                     [(p["threads"], round(p["decisions_per_s"]), round(p["p99_us"])) for p in sv.get("curve", [])]))
for k, v in (d.get("configs") or {}).items():
    print(k, "kernel_ms %.4f s2r_ms %.3f parity %s fu %s" % (v["kernel_ms"], v["submit_to_results_ms"], v["parity_sample"]["mismatches"],
                                                              v.get("device_followup_requests")))
print("reload", {k: v for k, v in (d.get("reload") or {}).items() if k != "c5_100k"}, (d.get("reload") or {}).get("c5_100k", {}).get("total_ms"))
print("cpu", (d.get("cpu_baseline") or {}).get("value"))
