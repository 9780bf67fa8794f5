#!/usr/bin/env python3
"""One small decode per mode with the per-kind launch profile (debug aid)."""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ldpc-simulator_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np
from ldpc_amd.device import Decoder, Graph
from conftest import hstd_for
code = sys.argv[1] if len(sys.argv) > 1 else "wimax_2304_0.5"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
T = int(sys.argv[3]) if len(sys.argv) > 3 else 5
H = hstd_for(code)
g = Graph.cached(H)
dec = Decoder(g, max(B, 64))
llr = np.random.default_rng(1).normal(2.0, 2.0, size=(B, H.shape[1]))
for mode in ("default", "tile", "split"):
    os.environ["LDPC_SMALL_COLS"] = "0" if mode != "default" else "32"
    dec.decode(llr, T, split=(mode == "split"))
    dec.profile(True)
    t0 = time.perf_counter()
    r = dec.decode(llr, T, split=(mode == "split"))
    dt = time.perf_counter() - t0
    p = dec.profile_read()
    dec.profile(False)
    print(json.dumps({"code": code, "B": B, "T": T, "mode": mode, "ms": round(dt * 1e3, 2),
                      "prof": {k: [round(v[0], 3), v[1]] for k, v in p.items() if v[1]}}), flush=True)
