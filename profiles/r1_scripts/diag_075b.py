"""Decode wimax_2304_0.75B once on the GPU through one path (argv[1]: split|tile)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("ldpc-simulator_amd", "tests", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
from conftest import hstd_for
from test_gpu_parity import _random_llr
from ldpc_amd.device import Decoder, Graph
H = hstd_for("wimax_2304_0.75B")
llr = _random_llr(H, 24, 4.0, seed=2408)
dec = Decoder(Graph(H), 24)
print("graph ok", flush=True)
r = dec.decode(llr, 8, nllr=True, post=True, hist=True, msgs=True, split=(sys.argv[1] == "split"))
print(sys.argv[1], "ok", r.conv.tolist(), flush=True)
