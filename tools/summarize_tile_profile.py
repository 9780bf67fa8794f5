#!/usr/bin/env python3
"""Summarize a tools/profile_tile.sh run into profiles/<tag>/ (committed evidence).

kernel_stats.csv  rocprofv3 --stats, verbatim
pmc_summary.csv   mean FETCH_SIZE / WRITE_SIZE per kernel (KiB as reported)
traffic.json      HBM bytes per launch of tile_kernel: FETCH_SIZE x 1024 x f +
                  WRITE_SIZE x 1024, f re-derived from the split path's
                  vn_kernel (reads each of nnz x frames messages once, 8 B).
usage: summarize_tile_profile.py SRC DST NNZ FRAMES
"""
import collections
import csv
import json
import os
import shutil
import sys


def mean_counter(path):
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in vals.items()}


def main(src, dst, nnz, frames):
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    fetch = mean_counter(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"))
    write = mean_counter(os.path.join(src, "pmc_write", "run_counter_collection.csv"))
    split = mean_counter(os.path.join(src, "pmc_fetch_split", "run_counter_collection.csv"))
    with open(os.path.join(dst, "pmc_summary.csv"), "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["run", "kernel", "dispatches", "FETCH_SIZE_KiB_mean", "WRITE_SIZE_KiB_mean"])
        for k in sorted(set(fetch) | set(write)):
            w.writerow(["tile", k, fetch.get(k, (0, 0))[1], fetch.get(k, (None,))[0], write.get(k, (None,))[0]])
        for k in sorted(split):
            w.writerow(["split", k, split[k][1], split[k][0], None])
    vn = max((k for k in split if "vn_kernel<" in k), key=lambda k: split[k][1])
    factor = 8.0 * nnz * frames / (split[vn][0] * 1024.0)
    def is_tile(k):  # tile_kernel (64 frames) or tile_sub_kernel<Q> (16 / 8 frames)
        return "tile_kernel" in k or "tile_sub_kernel" in k
    tk = max((k for k in fetch if is_tile(k)), key=lambda k: fetch[k][1])
    stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(dst, "kernel_stats.csv")))}
    st = next(v for n, v in stats.items() if is_tile(n))
    rd = fetch[tk][0] * 1024.0 * factor
    wr = write[tk][0] * 1024.0
    # frame-iterations one tile launch decoded (the traced bench line: one launch per step decodes
    # its `frames` frames, avg_iters each) -> bench.py scales the PMC bytes to its own run
    log = open(os.path.join(src, "bench_trace.log")).read()
    js = json.loads(log[log.index("{\"metric\""):].split("\n")[0])
    fi_launch = js["avg_iters"] * frames
    out = {"fetch_correction_factor": factor, "factor_source": vn, "frames": frames, "edges": nnz,
           "frame_iterations_per_launch": fi_launch,
           "kernels": {"tile": {"kernel": tk, "read_bytes": rd, "write_bytes": wr, "traffic_bytes": rd + wr,
                                "avg_ns": float(st["AverageNs"]), "calls": int(st["Calls"]),
                                "traffic_GBs": (rd + wr) / float(st["AverageNs"])}}}
    json.dump(out, open(os.path.join(dst, "traffic.json"), "w"), indent=2)
    print(json.dumps(out, indent=2))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
