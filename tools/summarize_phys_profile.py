#!/usr/bin/env python3
"""Summarize tools/profile_phys.sh into profiles/<tag>/ (committed evidence).

valu_snr<X>.json per SNR point: VALU wave-instructions per frame-iteration of
the physical-mode LDS decoder (SQ_INSTS_VALU summed over its dispatches /
frame-iterations of the same run), its VALU-busy share (SQ_ACTIVE_INST_VALU /
SQ_WAVE_CYCLES), and the issue roofline bench.py prices it against:
peak = 256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction
(MI355X_MICROARCH.md: v_fma_f32 wave64 throughput 2 cycles).
usage: summarize_phys_profile.py SRC DST
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

PEAK = 256 * 4 * 2.4e9 / 2.0


def sums(path, kfilter):
    agg, n = collections.defaultdict(float), collections.Counter()
    for r in csv.DictReader(open(path)):
        if kfilter in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]] += 1
    return agg, n


def bench_json(path):
    for line in open(path):
        if line.startswith("{"):
            return json.loads(line)
    raise ValueError(f"no bench JSON in {path}")


def one(src, dst, x):
    stats_src = glob.glob(os.path.join(src, f"trace_{x}", "**", "*kernel_stats.csv"), recursive=True)[0]
    shutil.copy(stats_src, os.path.join(dst, f"kernel_stats_snr{x}.csv"))
    b = bench_json(os.path.join(src, f"sq_{x}.log"))
    kname = b["roofline"]["kernel"]
    cc = glob.glob(os.path.join(src, f"sq_{x}", "**", "*counter_collection.csv"), recursive=True)[0]
    sq, n = sums(cc, kname)
    frames = b["config"]["frames_per_gpu"] * (b["steps"] + b["warmup"])
    fi = b["avg_iters"] * frames  # frame-iterations of the whole profiled run (warm-up included)
    stats = {r["Name"]: r for r in csv.DictReader(open(stats_src))}
    st = next(v for k, v in stats.items() if kname in k)
    total_s = float(st["TotalDurationNs"]) / 1e9
    out = {"kernel": kname, "code": b["config"]["code"], "snr_db": b["config"]["snr_db"],
           "avg_iters": b["avg_iters"], "frames_per_step": b["config"]["frames_per_gpu"],
           "dispatches": n["SQ_INSTS_VALU"], "frame_iterations": fi, "valu_insts": sq["SQ_INSTS_VALU"],
           "valu_insts_per_frame_iteration": sq["SQ_INSTS_VALU"] / fi,
           "valu_busy_share": sq["SQ_ACTIVE_INST_VALU"] / sq["SQ_WAVE_CYCLES"] if sq["SQ_WAVE_CYCLES"] else None,
           "wait_share": sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"] if sq["SQ_WAVE_CYCLES"] else None,
           "issue_stall_share": sq["SQ_WAIT_INST_ANY"] / sq["SQ_WAVE_CYCLES"] if sq["SQ_WAVE_CYCLES"] else None,
           "kernel_seconds_trace_run": total_s,
           "achieved_valu_insts_per_s_trace": sq["SQ_INSTS_VALU"] / total_s,
           "peak_valu_insts_per_s": PEAK, "frac": sq["SQ_INSTS_VALU"] / total_s / PEAK,
           "peak_model": "256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction"}
    json.dump(out, open(os.path.join(dst, f"valu_snr{x}.json"), "w"), indent=2)
    return out


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    xs = sorted(d[len("sq_"):] for d in os.listdir(src) if d.startswith("sq_") and not d.endswith(".log"))
    for x in xs:
        print(json.dumps(one(src, dst, x), indent=2))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
