"""One-line summary of a bench.py JSON line (for gpurun tails)."""
import json
import sys

d = json.loads([ln for ln in open(sys.argv[1]) if ln.startswith("{")][-1])
r = d.get("roofline") or {}
out = {"value": round(d["value"] or 0), "n_gpus": d.get("n_gpus"), "kernel": r.get("kernel"),
       "frac": round(r.get("frac", 0), 4), "avg_launch_ms": round(r.get("avg_launch_ms", 0), 1),
       "snr_points": [(p["snr_db"], p.get("scope", "step"), round(p["value"])) for p in d.get("snr_points", [])]}
ph = d.get("physical")
if ph:
    out["physical"] = (round(ph["value"]), round(ph.get("roofline", {}).get("frac", 0), 3), round(ph["avg_iters"], 2))
di = d.get("dropin")
if di:
    out["dropin_ms"] = round(di["ms_per_call"], 2)
cb = d.get("cpu_baseline")
if cb:
    out["cpu"] = (round(cb["value"], 2), cb["cores"])
print(json.dumps(out))
