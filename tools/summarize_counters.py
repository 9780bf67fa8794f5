#!/usr/bin/env python3
"""Summarize a counter breakdown (tools/profile_counters.sh) of one tile kernel.

usage: python tools/summarize_counters.py DIR KERNEL_SUBSTR FRAMES ITERS EDGES [OUT.json]

Reads DIR/<pass>/run_counter_collection.csv for every pass present, sums each
counter over the dispatches whose kernel name contains KERNEL_SUBSTR and
derives, per launch of FRAMES frames x ITERS iterations over EDGES H_std
edges (one "wave slot" = 64 lane-edges of one wavefront instruction):

  l2_hit_rate          TCC_HIT / (TCC_HIT + TCC_MISS)
  fabric_read_bytes    TCC_EA0_RDREQ x 128 B (every request 128 B: RDREQ_32B = 0;
                       2 x FETCH_SIZE, the guide's gfx950 halving)
  fabric_write_bytes   TCC_EA0_WRREQ x 64 B (all WRREQ_64B)
  read_x_algorithmic   fabric reads / (8 B x edges x frame-iterations)
  gather_miss_frac     (fabric read requests - E_old read requests) / L gather requests,
                       both at 128 B per request (a 16-frame lane group's 8 B each)
  sq_*_frac            SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY / _VALU over SQ_WAVE_CYCLES
  *_per_wave_slot      SQ_INSTS_* / wave slots
"""
import collections
import csv
import json
import os
import sys


def load(d, kern):
    agg = collections.defaultdict(float)
    n = collections.Counter()
    for p in sorted(os.listdir(d)):
        f = os.path.join(d, p, "run_counter_collection.csv")
        if not os.path.isfile(f):
            continue
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
                n[r["Counter_Name"]] += 1
    return agg, n


def main():
    d, kern, frames, iters, edges = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    agg, n = load(d, kern)
    if not agg:
        sys.exit(f"no dispatch of {kern!r} under {d}")
    launches = max(n.values())
    c = {k: v / n[k] for k, v in agg.items()}  # per launch
    efi = float(edges) * frames * iters
    slots = efi / 64.0
    alg_read = 8.0 * efi
    out = {"dir": d, "kernel": kern, "frames": frames, "iters": iters, "edges": edges, "launches_per_pass": launches,
           "counters_per_launch": c}
    if "TCC_HIT_sum" in c:
        out["l2_hit_rate"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    if "TCC_EA0_RDREQ_sum" in c:
        rd = c["TCC_EA0_RDREQ_sum"] * 128.0
        out["fabric_read_bytes"] = rd
        out["read_x_algorithmic"] = rd / alg_read
        eold_req = alg_read / 128.0  # E_old: 8 B x 16 frames of a lane group = one 128-B request
        gather_req = alg_read / 128.0
        out["gather_miss_frac"] = (c["TCC_EA0_RDREQ_sum"] - eold_req) / gather_req
    if "TCC_EA0_WRREQ_sum" in c:
        out["fabric_write_bytes"] = c["TCC_EA0_WRREQ_sum"] * 64.0
        out["write_x_algorithmic"] = out["fabric_write_bytes"] / alg_read
    if "SQ_WAVE_CYCLES" in c:
        w = c["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS"):
            if k in c:
                out[k.lower().replace("sq_", "sq_") + "_frac"] = c[k] / w
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
              "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH", "SQ_LDS_BANK_CONFLICT"):
        if k in c:
            out[k.lower() + "_per_wave_slot"] = c[k] / slots
    s = json.dumps(out, indent=1)
    if len(sys.argv) > 6:
        open(sys.argv[6], "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
