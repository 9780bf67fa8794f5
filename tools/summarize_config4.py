#!/usr/bin/env python3
"""Summarize tools/profile_config4.sh into profiles/<tag>/ (committed evidence):
kernel_stats_{sweep,static}.csv (rocprofv3 --stats) and traffic.json --
HBM bytes from FETCH_SIZE / WRITE_SIZE (KiB), reads corrected by the gfx950
factor calibrated on the SAME access width: the r3/4 graphs keep E in 8-frame
blocks (64 B per lane group, as the L gather of 8 frames), and vn_kernel on
that layout -- each message read once -- gives 1.010
(profiles/r3b_tile8_r34_prof/summary.json); the 1.986 of the 16-frame/128-B
layout (profiles/r3p_final, MI355X_MICROARCH.md: FETCH_SIZE tallies 64 B per
128-B request) does not apply here:
  kernels.tile8_stream: the whole sweep (every kernel of the sweep process:
      frame order, tile8_stream_kernel, the split tail, compaction), bytes
      for the sweep -- bench.py's config4 roofline scope;
  kernels.tile: the static 1 dB step's tile8_kernel, bytes per launch.
usage: summarize_config4.py SRC DST
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

FACTOR = 1.0100041410403928  # profiles/r3b_tile8_r34_prof/summary.json (vn_kernel<false, true>, 8-frame E blocks)


def one(path):
    return glob.glob(os.path.join(path, "**", "*.csv"), recursive=True)


def counters(src, mode, name):
    f = [p for p in one(os.path.join(src, f"{mode}_{name}")) if p.endswith("counter_collection.csv")][0]
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return per


def bench_line(path):
    for ln in open(path):
        if ln.startswith("{"):
            return json.loads(ln)
    raise ValueError(path)


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    out = {"fetch_correction_factor": FACTOR, "factor_source": "profiles/r3b_tile8_r34_prof/summary.json (vn_kernel on 8-frame E blocks)",
           "kernels": {}}
    for mode in ("sweep", "static"):
        st = [p for p in one(os.path.join(src, f"{mode}_trace")) if p.endswith("kernel_stats.csv")][0]
        shutil.copy(st, os.path.join(dst, f"kernel_stats_{mode}.csv"))
        info = bench_line(os.path.join(src, f"{mode}_trace.log"))
        fe, wr = counters(src, mode, "fetch"), counters(src, mode, "write")
        rd_all = sum(sum(v) for v in fe.values()) * 1024.0 * FACTOR
        wr_all = sum(sum(v) for v in wr.values()) * 1024.0
        out["edges"], out["n"] = info["edges"], info["n"]
        if mode == "sweep":
            out["frames"] = info["slots"]
            out["kernels"]["tile8_stream"] = {
                "scope": "whole sweep, every kernel of the sweep process", "points": info["points"],
                "read_bytes": rd_all, "write_bytes": wr_all, "traffic_bytes": rd_all + wr_all,
                "algorithmic_bytes": sum(p["frames"] * (8 * info["n"] + (info["n"] + 7) // 8 + 8)
                                         + 16.0 * info["edges"] * p["iters"] for p in info["points"]),
                "per_kernel_bytes": {k: sum(fe[k]) * 1024.0 * FACTOR + sum(wr.get(k, [0.0])) * 1024.0 for k in fe}}
        else:
            k = next(k for k in fe if "tile8_kernel" in k)
            rd, w = sum(fe[k]) / len(fe[k]) * 1024.0 * FACTOR, sum(wr[k]) / len(wr[k]) * 1024.0
            p = info["points"][0]
            out["static"] = {"frames": info["frames"], "edges": info["edges"]}
            out["kernels"]["tile"] = {"kernel": k, "read_bytes": rd, "write_bytes": w, "traffic_bytes": rd + w,
                                      "algorithmic_bytes": p["frames"] * (8 * info["n"] + (info["n"] + 7) // 8 + 8)
                                      + 16.0 * info["edges"] * p["iters"]}
    # bench.py committed_traffic() keys on (edges, frames): the sweep's slots here;
    # the static step's entry goes to a second file keyed on its 32,768 frames
    st = {"fetch_correction_factor": FACTOR, "edges": out["edges"], "frames": out["static"]["frames"],
          "kernels": {"tile": out["kernels"].pop("tile")}}
    json.dump(out, open(os.path.join(dst, "traffic.json"), "w"), indent=2)
    json.dump(st, open(os.path.join(dst, "traffic_static.json"), "w"), indent=2)
    print(json.dumps(out, indent=2)[:3000])
    print(json.dumps(st, indent=2))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
