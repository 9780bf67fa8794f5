"""Bitwise A/B of two builds of libldpc_hip.so (GPU box): decode the same
seeded batches with each (one child process per library, LDPC_HIP_LIB) and
require identical z / conv / status / iters / posteriors / messages.
usage: python tools/compare_libs.py variants/a.so variants/b.so"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [("wimax_576_0.5", 256, 0.0, 20, False), ("wimax_576_0.5", 256, 2.0, 30, False),
         ("wimax_576_0.5", 192, 1.0, 12, True), ("wimax_2304_0.75A", 64, 3.0, 8, False),
         ("BCH_7_4_1_strip", 640, 1.0, 10, False)]

if len(sys.argv) == 4 and sys.argv[1] == "--child":
    sys.path.insert(0, os.path.join(ROOT, "ldpc-simulator_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from conftest import hstd_for
    from test_gpu_parity import _random_llr
    from ldpc_amd.device import Decoder, Graph
    out = {}
    for ci, (code, B, snr, T, split) in enumerate(CASES):
        H = hstd_for(code)
        llr = _random_llr(H, B, snr, seed=900 + ci)
        r = Decoder(Graph(H), B).decode(llr, T, nllr=True, post=True, msgs=True, split=split)
        for k in ("z", "conv", "status", "iters", "post", "msgs", "nllr"):
            out[f"{ci}_{k}"] = r[k]
    np.savez(sys.argv[3], **out)
    sys.exit(0)

res = []
for i, lib in enumerate(sys.argv[1:3]):
    f = f"/tmp/cmp_{i}.npz"
    subprocess.run([sys.executable, __file__, "--child", lib, f], check=True,
                   env=dict(os.environ, LDPC_HIP_LIB=lib), timeout=300)
    res.append(np.load(f))
bad = [k for k in res[0].files if not np.array_equal(res[0][k], res[1][k])]
print("identical" if not bad else f"DIFFER: {bad}", f"({len(res[0].files)} arrays, {len(CASES)} cases)")
sys.exit(1 if bad else 0)
