#!/usr/bin/env python3
"""Per-call latency of Decoder.decode on small batches of wimax_2304_0.5
(T=50, ~1 dB) under environment variants given as NAME=VAL[,NAME=VAL] args
('-' = default).  One JSON line per (variant, B)."""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ldpc-simulator_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np
from ldpc_amd.device import Decoder, Graph
from conftest import hstd_for

code = os.environ.get("CODE", "wimax_2304_0.5")
H = hstd_for(code)
m, n = H.shape
g = Graph.cached(H)
rng = np.random.default_rng(1)
Bs = [int(b) for b in os.environ.get("BS", "1,64,256,1024").split(",")]
for B in Bs:
    dec = Decoder(g, max(B, 64))
    llr = rng.normal(float(os.environ.get("MEAN", "2.0")), 2.0, size=(B, n))
    ref = None
    for var in sys.argv[1:]:
        keys = []
        if var != "-":
            for kv in var.split(","):
                k, v = kv.split("=")
                os.environ[k] = v
                keys.append(k)
        dec.decode(llr, 50)
        t0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            r = dec.decode(llr, 50)
        dt = (time.perf_counter() - t0) / reps
        same = None
        if ref is None:
            ref = r
        else:
            same = bool(np.array_equal(r.z, ref.z) and np.array_equal(r.conv, ref.conv))
        print(json.dumps({"code": code, "B": B, "var": var, "ms_per_call": round(dt * 1e3, 2),
                          "cw_s": round(B / dt, 1), "iters_mean": float(np.mean(r.iters)), "same_as_first": same}),
              flush=True)
        for k in keys:
            os.environ.pop(k)
    dec.close()
