"""Probe: torch (its bundled HIP runtime) and libldpc_hip.so (linked against
/opt/rocm's) in one process, in either initialisation order.  Both libraries
carry the soname libamdhip64.so.7, so the first one loaded serves both.
usage: python tools/runtime_order_probe.py torch-first|lib-first"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ldpc-simulator_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def lib_decode():
    from ldpc_amd.device import Decoder, Graph
    from conftest import hstd_for
    H = hstd_for("wimax_576_0.5")
    dec = Decoder(Graph.cached(H), 64)
    rng = np.random.default_rng(1)
    r = dec.decode(rng.normal(2.0, 2.0, (64, H.shape[1])), 5)
    return int(r.conv.sum())


def torch_op():
    import torch
    x = torch.arange(8, dtype=torch.float64, device="cuda:0")
    return float((x * 2).sum().item()), torch.cuda.device_count()


order = sys.argv[1]
if order == "torch-first":
    print("torch", torch_op(), flush=True)
    print("lib", lib_decode(), flush=True)
    print("torch again", torch_op(), flush=True)
else:
    print("lib", lib_decode(), flush=True)
    print("torch", torch_op(), flush=True)
    print("lib again", lib_decode(), flush=True)
import ctypes  # noqa: E402
for name in ("libamdhip64.so.7",):
    print("loaded:", [l for l in open("/proc/self/maps").read().split("\n") if "libamdhip64" in l][:1], flush=True)
print("ok", order, flush=True)
