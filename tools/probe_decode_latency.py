#!/usr/bin/env python3
"""Per-call latency of Decoder.decode on small batches (the drop-in per-frame
path): wimax_2304_0.5 / 0.75A at 1 dB, T=50, batch B in 1, 16, 64, 256, 1024,
with the default policy and with LDPC_SMALL_COLS=0 (the tile decoders).
Prints one JSON line per (code, B, mode)."""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ldpc-simulator_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np
from ldpc_amd.device import Decoder, Graph
from conftest import hstd_for

for code in ("wimax_2304_0.5", "wimax_2304_0.75A"):
    H = hstd_for(code)
    m, n = H.shape
    g = Graph.cached(H)
    rng = np.random.default_rng(1)
    for B in (1, 16, 64, 256, 1024):
        dec = Decoder(g, max(B, 64))
        llr = rng.normal(2.0, 2.0, size=(B, n))  # all-zero codeword at roughly 1 dB (LLR mean 2/sigma^2 ~ 2)
        for mode in ("default", "tile"):
            if mode == "tile":
                os.environ["LDPC_SMALL_COLS"] = "0"
            else:
                os.environ.pop("LDPC_SMALL_COLS", None)
            dec.decode(llr, 50)  # warm-up
            t0 = time.perf_counter()
            reps = 3
            for _ in range(reps):
                r = dec.decode(llr, 50)
            dt = (time.perf_counter() - t0) / reps
            print(json.dumps({"code": code, "B": B, "mode": mode, "ms_per_call": round(dt * 1e3, 2),
                              "cw_s": round(B / dt, 1), "iters_mean": float(np.mean(r.iters))}), flush=True)
        dec.close()
