#!/usr/bin/env python3
"""Summarize tools/profile_phys.sh into profiles/<tag>/ (committed evidence).

valu.json: VALU wave-instructions per frame-iteration of the physical-mode LDS
decoder (SQ_INSTS_VALU summed over its dispatches / frame-iterations of the
same run), its VALU-busy share (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES, both
quad-cycle counts), and the issue roofline bench.py prices it against:
peak = 256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction
(MI355X_MICROARCH.md: v_fma_f32 wave64 throughput 2 cycles).
usage: summarize_phys_profile.py SRC DST
"""
import collections
import csv
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


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "phys_trace", "run_kernel_stats.csv"), os.path.join(dst, "phys_kernel_stats.csv"))
    shutil.copy(os.path.join(src, "tail_trace", "run_kernel_stats.csv"), os.path.join(dst, "tail_3dB_kernel_stats.csv"))
    b = bench_json(os.path.join(src, "phys_sq.log"))
    kname = b["roofline"]["kernel"]
    sq, n = sums(os.path.join(src, "phys_sq", "run_counter_collection.csv"), kname)
    frames = b["config"]["frames_per_gpu"] * (b["steps"] + b["warmup"])
    fi = b["avg_iters"] * frames  # frame-iterations of the whole profiled run
    stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(dst, "phys_kernel_stats.csv")))}
    st = next(v for k, v in stats.items() if kname in k)
    total_s = float(st["TotalDurationNs"]) / 1e9
    out = {"kernel": kname, "code": b["config"]["code"], "snr_db": b["config"]["snr_db"],
           "frames_per_step": b["config"]["frames_per_gpu"], "dispatches": n["SQ_INSTS_VALU"],
           "frame_iterations": fi, "valu_insts": sq["SQ_INSTS_VALU"],
           "valu_insts_per_frame_iteration": sq["SQ_INSTS_VALU"] / fi,
           "valu_busy_share": sq["SQ_ACTIVE_INST_VALU"] / sq["SQ_WAVE_CYCLES"] if sq["SQ_WAVE_CYCLES"] else None,
           "wait_share": sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"] if sq["SQ_WAVE_CYCLES"] else None,
           "issue_stall_share": sq["SQ_WAIT_INST_ANY"] / sq["SQ_WAVE_CYCLES"] if sq["SQ_WAVE_CYCLES"] else None,
           "kernel_seconds_trace_run": total_s,
           "achieved_valu_insts_per_s_trace": sq["SQ_INSTS_VALU"] / total_s,
           "peak_valu_insts_per_s": PEAK, "frac": sq["SQ_INSTS_VALU"] / total_s / PEAK,
           "peak_model": "256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction"}
    json.dump(out, open(os.path.join(dst, "valu.json"), "w"), indent=2)
    t = bench_json(os.path.join(src, "tail_bench.json"))
    json.dump(t, open(os.path.join(dst, "tail_3dB_bench.json"), "w"))
    print(json.dumps(out, indent=2))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
