#!/usr/bin/env python3
"""Summarize a tools/gpu_prof3.sh run into profiles/<tag>/ (committed evidence).

kernel_stats.csv  rocprofv3 --stats of the T=50 bench, verbatim
summary.json      per launch of the decoder kernel: HBM read bytes (FETCH_SIZE x
                  1 KiB x f, f re-derived from the split path's vn_kernel, which
                  reads each of nnz x frames messages once), write bytes
                  (WRITE_SIZE x 1 KiB), bytes per edge-frame-iteration, and the
                  SQ-counter readings of the T=10 run (VALU busy, wait fraction,
                  instructions per wavefront edge slot).
usage: summarize_prof3.py SRC DST NNZ FRAMES ITERS FRAMES_PER_SLOT
  FRAMES_PER_SLOT: frames one wavefront instruction covers per edge
  (tile_sub: 16 = 4 edges x 16 frames per 64 lanes; tile8: 8 = 8 edges x 8 frames)
"""
import collections, csv, glob, json, os, shutil, sys


def counters(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Kernel_Name"]].add(r["Dispatch_Id"])
    return vals, disp


def is_dec(k):
    return any(s in k for s in ("tile_kernel", "tile_sub_kernel", "tile8_kernel"))


def main(src, dst, nnz, frames, iters, fps):
    nnz, frames, iters, fps = int(nnz), int(frames), int(iters), int(fps)
    os.makedirs(dst, exist_ok=True)
    ks = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)[0]
    shutil.copy(ks, os.path.join(dst, "kernel_stats.csv"))
    stats = {r["Name"]: r for r in csv.DictReader(open(ks))}
    name = next(n for n in stats if is_dec(n))
    fetch, fd = counters(os.path.join(src, "fetch"))
    write, wd = counters(os.path.join(src, "write"))
    split, sd = counters(os.path.join(src, "fetch_split"))
    vn = max((k for k in split if "vn_kernel<" in k), key=lambda k: len(sd[k]))
    f = 8.0 * nnz * frames * len(sd[vn]) / (split[vn]["FETCH_SIZE"] * 1024.0)
    dk = next(k for k in fetch if is_dec(k))
    n = len(fd[dk])
    rd = fetch[dk]["FETCH_SIZE"] * 1024.0 * f / n
    wr = write[dk]["WRITE_SIZE"] * 1024.0 / len(wd[dk])
    efi = float(nnz) * frames * iters
    out = {"kernel": dk, "avg_ms": float(stats[name]["AverageNs"]) / 1e6, "calls": int(stats[name]["Calls"]),
           "fetch_correction_factor": f, "factor_source": vn,
           "read_bytes_per_launch": rd, "write_bytes_per_launch": wr, "traffic_bytes_per_launch": rd + wr,
           "bytes_per_edge_frame_iteration": (rd + wr) / efi, "algorithmic_bytes_per_edge_frame_iteration": 16.0,
           "edges": nnz, "frames": frames, "iterations": iters}
    sq1, s1 = counters(os.path.join(src, "sq1"))
    sq2, s2 = counters(os.path.join(src, "sq2"))
    k1 = next(k for k in sq1 if is_dec(k))
    k2 = next(k for k in sq2 if is_dec(k))
    a, b = sq1[k1], sq2[k2]
    slots = float(nnz) * frames * 10 / 64.0  # wavefront edge slots at T=10 (64 lanes)
    grbm_per_xcd = a["GRBM_GUI_ACTIVE"] / 8.0
    out["sq_T10"] = {
        "SQ": {**a, **b},
        "valu_busy_fraction": a["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * grbm_per_xcd),
        "wave_wait_fraction": a["SQ_WAIT_ANY"] / a["SQ_WAVE_CYCLES"],
        "valu_per_wave_edge_slot": a["SQ_INSTS_VALU"] / slots,
        "salu_per_wave_edge_slot": a["SQ_INSTS_SALU"] / slots,
        "lds_per_wave_edge_slot": b["SQ_INSTS_LDS"] / slots,
        "lds_bank_conflict_fraction": b["SQ_LDS_BANK_CONFLICT"] / max(b["SQ_LDS_IDX_ACTIVE"], 1.0),
        "lds_busy_fraction": b["SQ_LDS_IDX_ACTIVE"] / (256 * grbm_per_xcd),
        "slot_definition": "one wavefront instruction over 64 lanes = %d edges x %d frames" % (64 // fps, fps),
    }
    json.dump(out, open(os.path.join(dst, "summary.json"), "w"), indent=1)
    # bench.py committed_traffic(): HBM bytes per launch of this exact shape
    json.dump({"edges": nnz, "frames": frames, "source": "summary.json (this directory)",
               "kernels": {"tile": {"kernel": dk, "traffic_bytes": rd + wr, "read_bytes": rd, "write_bytes": wr,
                                    "avg_ns": out["avg_ms"] * 1e6}}},
              open(os.path.join(dst, "traffic.json"), "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "sq_T10"}, indent=1))
    print(json.dumps({k: v for k, v in out["sq_T10"].items() if k != "SQ"}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:7])
