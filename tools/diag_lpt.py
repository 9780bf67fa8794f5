"""Diagnostic (GPU): how early the streaming supply order (frame_order.hip)
starts the frames that fail, on one 32,768-frame point of wimax_2304_0.5.
Prints the supply positions of the failing frames (fraction of the point) and
a slot-level model of the step: 4,096 slots, a frame takes its iteration
count of passes, the tail (after the supply is out) costs `ctail` of a pass
per iteration.  usage: python tools/diag_lpt.py [snr] [frames]"""
import heapq
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ldpc-simulator_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle  # noqa: E402
from conftest import hstd_for  # noqa: E402
from ldpc_amd.device import Decoder, Graph  # noqa: E402

snr = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
N = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
code = "wimax_2304_0.5"
H = hstd_for(code)
sig = oracle.sigma_for_snr(snr)
seed, point, frame0 = 20240601, 3, 0
dec = Decoder(Graph(H), 4096)
order = dec.frame_order(seed, point, sig, frame0, N)
its = np.empty(N, np.int32)
fail = np.empty(N, bool)
for a in range(0, N, 4096):
    _, llr = dec.generate(seed, point, sig, frame0 + a, min(4096, N - a))
    r = dec.decode(llr, 50)
    its[a:a + len(llr)] = r.iters
    fail[a:a + len(llr)] = r.status != 0
pos = np.empty(N, np.int64)
pos[order] = np.arange(N)
print(f"{code} {snr} dB, {N} frames: failing {fail.sum()}, avg iterations {its.mean():.2f}")
print("supply positions of failing frames (fraction):", np.round(np.sort(pos[fail]) / N, 3)[-12:])


def model(o, slots=4096, ctail=0.54):
    heap = [(0.0, s) for s in range(slots)]
    ends = []
    for f in o:
        t, s = heapq.heappop(heap)
        heapq.heappush(heap, (t + its[f], s))
        ends.append((t, t + its[f]))
    se = max(a for a, _ in ends)
    tl = max(b for _, b in ends) - se
    return se, tl, se + ctail * tl


for name, o in (("device order", order), ("index order", np.arange(N)), ("by iterations", np.argsort(-its, kind="stable"))):
    print("%-14s supply %5.1f passes, tail %5.1f, total %6.1f" % ((name,) + model(o)))

# the failing frames the order starts late: what the receiver saw
Hc = H.tocsr()
m, n = Hc.shape
k = n - m
odd = (np.diff(Hc.indptr) % 2) == 1
late = np.where(fail & (pos > 0.1 * N))[0]
for f in late[:12]:
    _, l1 = dec.generate(seed, point, sig, frame0 + int(f), 1)
    l1 = l1[0]
    hard = (l1 > 0).astype(np.int64)
    syn = int(((Hc @ hard) % 2).sum())
    a = np.abs(l1)
    print(f"late failing frame {f}: pos {pos[f] / N:.3f} iters {its[f]} syn {syn} minI_odd {a[k:][odd].min():.3f} "
          f"minI_even {a[k:][~odd].min():.3f} minA {a[:k].min():.4f} neg-bits {int((l1 < 0).sum())}")
