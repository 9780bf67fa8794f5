"""One-line summary of a bench.py JSON line (for gpurun tails)."""
import json
import sys

d = json.loads([ln for ln in open(sys.argv[1]) if ln.startswith("{")][-1])
r = d.get("roofline") or {}
dr = d.get("decode_roofline") or {}
out = {"value": round(d["value"] or 0), "ms": {k[:-3]: round(v) for k, v in dr.items() if k.endswith("_ms") and v}, "n_gpus": d.get("n_gpus"), "kernel": r.get("kernel"),
       "frac": round(r.get("frac", 0), 4), "avg_launch_ms": round(r.get("avg_launch_ms", 0), 1),
       "snr_points": [(p["snr_db"], p.get("scope", "step"), round(p["value"])) for p in d.get("snr_points", [])]}
ph = d.get("physical")
if ph:
    out["physical"] = (round(ph["value"]), round(ph.get("roofline", {}).get("frac", 0), 3), round(ph["avg_iters"], 2))
if ph and ph.get("waterfall"):
    w = ph["waterfall"]
    out["phys_waterfall"] = (round(w["value"]), round(w.get("roofline", {}).get("frac", 0), 3), round(w["avg_iters"], 2))
c4 = d.get("config4")
if c4:
    out["config4"] = (round(c4["value"]), round(c4["roofline"]["frac"], 3),
                      [(p["snr_db"], round(p["value"]), round(p["roofline_frac"] or 0, 3)) for p in c4["points"]])
    s4 = c4.get("static_1dB") or {}
    out["config4_static"] = (round(s4.get("value", 0)), round((s4.get("roofline") or {}).get("frac", 0), 3))
for key in ("config2", "config5"):
    c = d.get(key)
    if c:
        out[key] = (round(c["value"]), round((c.get("roofline") or {}).get("frac", 0), 3), round(c["avg_iters"], 2))
di = d.get("dropin")
if di:
    out["dropin_ms"] = round(di["ms_per_call"], 2)
cb = d.get("cpu_baseline")
if cb:
    out["cpu"] = (round(cb["value"], 2), cb["cores"])
print(json.dumps(out))
