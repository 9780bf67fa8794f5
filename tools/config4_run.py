#!/usr/bin/env python3
"""BASELINE config 4 alone, for profiling (tools/profile_config4.sh): the bench's
config4 sweep (wimax_2304_0.75A, 1.0:0.5:4.0 dB, 32,768 frames per point through
2,048 streaming slots: tile8_stream_kernel + the split tail) with `sweep`, or its
static 1 dB step (one tile8_kernel launch over 32,768 frames) with `static`.
Same calls, seeds and frame ranges as bench.py config4_extra.  Prints one JSON
line: counters and frame-iterations per point (for the byte model)."""
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ldpc-simulator_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402  (SEED, snr_grid)
import ldpc_amd  # noqa: E402
from ldpc_amd.device import Decoder, Graph  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "sweep"
F, SLOTS, T = 32768, 2048, 50
edd = ldpc_amd.load_committed_code("wimax_2304_0.75A")
g = Graph(edd._h_std)
sig = lambda x: 1.0 / math.sqrt(2.0 * (10.0 ** (x * 0.1)))  # noqa: E731
base = 1 << 43
out = {"mode": mode, "edges": int(edd._h_std.nnz), "n": edd._n, "frames": F, "points": []}
if mode == "sweep":
    dec = Decoder(g, SLOTS)
    out["slots"] = SLOTS
    for i, x in enumerate(bench.snr_grid("1.0:0.5:4.0")):
        c = dec.mc_run(bench.SEED, [sig(x)], F, base + i * F, T)
        out["points"].append({"snr_db": x, "frames": int(c[0, 0]), "iters": int(c[0, 6])})
else:
    dec = Decoder(g, F)
    c = dec.mc_run(bench.SEED, [sig(1.0)], F, base + (1 << 40), T, static=True)
    out["points"].append({"snr_db": 1.0, "frames": int(c[0, 0]), "iters": int(c[0, 6])})
print(json.dumps(out), flush=True)
