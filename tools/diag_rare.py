"""Diagnostic (GPU): where the tile decoders and the split path part on
exact-zero channel LLRs (tests/test_gpu_decoders.py::test_2304_rare_rows)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ldpc-simulator_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle  # noqa: E402
from conftest import hstd_for  # noqa: E402
from test_gpu_parity import _random_llr  # noqa: E402
from ldpc_amd.device import Decoder, Graph  # noqa: E402

code = "wimax_2304_0.5"
H = hstd_for(code)
B = 24
llr = _random_llr(H, B, 2.0, seed=77)
rng = np.random.default_rng(78)
for f in range(B):
    llr[f, rng.choice(H.shape[1], size=1 + f % 4, replace=False)] = 0.0
frames = [2, 15]
g = Graph(H)
for T in range(1, 6):
    os.environ["LDPC_SMALL_COLS"] = "0"
    dt = Decoder(g, B)
    rt = dt.decode(llr, T, post=True, msgs=True)
    rs = dt.decode(llr, T, split=True, post=True, msgs=True)
    o = oracle.spa_decode(H, llr, T, want_E=True)
    for f in frames:
        dL = np.nonzero(rt.post[f] != rs.post[f])[0]
        dE = np.nonzero(rt.msgs[f] != rs.msgs[f])[0]
        oL = np.nonzero(rs.post[f] != o["post"][f])[0]
        print(f"T={T} f={f}: tile!=split L at {dL[:8]} ({dL.size}), E at {dE[:8]} ({dE.size}); split!=oracle L {oL.size};"
              f" z tile/split/oracle {rt.z[f][dL[:3]] if dL.size else ''} {rs.z[f][dL[:3]] if dL.size else ''}")
        for c in dL[:3]:
            print(f"    col {c}: tile {rt.post[f][c]!r} split {rs.post[f][c]!r} oracle {o['post'][f][c]!r} ch {llr[f][c]!r}")
        for e in dE[:4]:
            print(f"    edge {e}: tile {rt.msgs[f][e]!r} split {rs.msgs[f][e]!r} oracle {o['msgs'][f][e]!r}")
