#!/usr/bin/env python3
"""Timeline of tile_kernel's phases from a -DLDPC_TILE_TRACE build (GPU box):
  LDPC_HIP_LIB=variants/trace.so python tools/tile_trace.py
Stamps (s_memtime, shader cycles) per wavefront w and row r of pass 2 in
workgroup 0: 0 P3 start, 1 final product acquired, 2 P3 end, 3 hop wait start,
4 hop wait end, 5 hop published, 6 P1 end (row r = the row P1 loaded)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("ldpc-simulator_amd", "tests", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import oracle  # noqa: E402
from conftest import hstd_for  # noqa: E402
from ldpc_amd import _lib  # noqa: E402
from ldpc_amd.device import Decoder, Graph  # noqa: E402

W, R, EV = 16, 64, 8
frames = int(os.environ.get("FRAMES", "16384"))
dec = Decoder(Graph(hstd_for("wimax_576_0.5")), frames)
sig = [oracle.sigma_for_snr(0.0)]
dec.mc_run(20260213, sig, frames, 0, 6, static=True)  # warm-up
dec.mc_run(20260213, sig, frames, 0, 6, static=True)
buf = (ctypes.c_uint64 * (W * R * EV))()
n = _lib.lib().ldpc_diag_tile_trace(buf, W * R * EV)
if n < 0:
    raise SystemExit("not a trace build")
t = np.frombuffer(buf, dtype=np.uint64).reshape(W, R, EV).astype(np.int64)
rows = range(2, R - 2)


def stat(name, v):
    v = np.asarray(v, np.float64)
    print(f"{name:44s} mean {v.mean():8.0f}  median {np.median(v):8.0f}  p90 {np.percentile(v, 90):8.0f}")


final = t[W - 1, :, 5]
stat("row period final(r+1)-final(r)", [final[r + 1] - final[r] for r in rows])
stat("chain: hop published w15 - w0 (same row)", [t[W - 1, r, 5] - t[0, r, 5] for r in rows])
stat("per hop (w-1 published -> w published)", [t[w, r, 5] - t[w - 1, r, 5] for r in rows for w in range(1, W)])
stat("hop wait (stamp 4 - 3)", [t[w, r, 4] - t[w, r, 3] for r in rows for w in range(1, W)])
stat("hop work after wait (5 - 4)", [t[w, r, 5] - t[w, r, 4] for r in rows for w in range(1, W)])
stat("P3 wait for final (1 - 0)", [t[w, r, 1] - t[w, r, 0] for r in rows for w in range(W)])
stat("P3 work (2 - 1)", [t[w, r, 2] - t[w, r, 1] for r in rows for w in range(W)])
stat("final(r) -> w0 hop(r+1) published", [t[0, r + 1, 5] - final[r] for r in rows])
stat("final(r) -> w P3(r) end", [t[w, r, 2] - final[r] for r in rows for w in range(W)])
stat("P1(r+2) (6[r+2] - 5[r+1])", [t[w, r + 2, 6] - t[w, r + 1, 5] for r in rows for w in range(W)])
stat("wave busy P3+P1 per row", [(t[w, r, 2] - t[w, r, 1]) + (t[w, r + 2, 6] - t[w, r + 1, 5]) for r in rows for w in range(W)])
np.save(os.path.join(ROOT, "gpurun_out", "tile_trace.npy"), t)
