#!/usr/bin/env python3
"""BER/FER curve of the GPU decoder overlaid on the reference's own curve
(north_star: "BER curve overlaying the CPU reference at Eb/N0 1.0-3.0 dB").

The reference curve (tests/golden/ber_curve_wimax_576_0.5.json) was measured by
running the reference's main.py (tests/golden/gen_ber_curve.py): its channel
and generator are time-seeded MT19937, so the overlay is statistical.  For
each SNR point the GPU decodes G groups of exactly the reference's frame count
B (on-device frames, Philox-keyed by frame index, same channel model), giving
the sampling distribution of FER and BER at that sample size; the reference's
value must fall inside its central 99 % (deterministic: the reference numbers
are fixed and the GPU frames are seeded).  Per-frame outcomes follow main.py
(:130-138): a frame fails iff its syndrome is non-zero after the last
iteration, and BER counts u != z^1 bits of failed frames only.

Run on the GPU box:  python tests/ber_overlay.py [code]   (prints the overlay table)
Reference curves: wimax_576_0.5 (5 points, 96-384 frames each) and the
north-star code wimax_2304_0.5 (1.0 / 2.0 / 3.0 dB, 8 / 80 / 64 frames: a 2304
frame-iteration costs the reference ~25 s of one core; the 2 dB point, the only
one off the curve's floors, is two runs of the reference summed: 16 + 64
frames, gen_ber_curve.py --append).
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(ROOT, "ldpc-simulator_amd"), HERE, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

REF_FMT = os.path.join(HERE, "golden", "ber_curve_{}.json")
SEED = 20260213
GROUPS = 400


def load_reference(code="wimax_576_0.5"):
    return json.load(open(REF_FMT.format(code)))


def gpu_groups(dec, snr_db, B, G, max_iter, seed=SEED, snr_point=0):
    """Per-group (failed, err_bits) over G groups of B on-device frames."""
    import oracle
    k = dec.graph.k
    sigma = oracle.sigma_for_snr(snr_db)
    total = B * G
    failed = np.zeros(total, np.int64)
    err = np.zeros(total, np.int64)
    chunk = (dec.capacity // B) * B
    for s in range(0, total, chunk):
        c = min(chunk, total - s)
        u, llr = dec.generate(seed, snr_point, sigma, s, c)
        r = dec.decode(llr, max_iter)
        bad = r.status != 0
        failed[s:s + c] = bad
        e = np.count_nonzero(u.astype(np.uint8) != (r.z[:, :k] ^ 1), axis=1)
        err[s:s + c] = np.where(bad, e, 0)
    return failed.reshape(G, B).sum(1), err.reshape(G, B).sum(1)


def overlay(dec, ref=None, groups=GROUPS, q=0.005, code="wimax_576_0.5"):
    """One row per reference point: reference FER/BER, the GPU's pooled values
    and the [q, 1-q] quantiles of its group FER/BER at the reference's B."""
    ref = ref or load_reference(code)
    k = dec.graph.k
    T = int(ref["max_iter"])
    rows = []
    for i, p in enumerate(ref["points"]):
        B = int(p["blocks"])
        fg, eg = gpu_groups(dec, float(p["snr_db"]), B, groups, T, snr_point=i)
        fer_g, ber_g = fg / B, eg / (k * B)
        rows.append({
            "snr_db": p["snr_db"], "B": B, "groups": groups,
            "fer_ref": p["failed"] / B, "ber_ref": p["err_bits"] / (k * B),
            "fer_gpu": float(fer_g.mean()), "ber_gpu": float(ber_g.mean()),
            "fer_lo": float(np.quantile(fer_g, q)), "fer_hi": float(np.quantile(fer_g, 1 - q)),
            "ber_lo": float(np.quantile(ber_g, q)), "ber_hi": float(np.quantile(ber_g, 1 - q)),
        })
    return rows


def main():
    import ldpc_amd
    from conftest import hstd_for
    from ldpc_amd.device import Decoder, Graph
    if ldpc_amd.device_count() <= 0:
        raise SystemExit("needs a GPU")
    code = sys.argv[1] if len(sys.argv) > 1 else "wimax_576_0.5"
    dec = Decoder(Graph(hstd_for(code)), 16384)
    rows = overlay(dec, code=code)
    print("| SNR dB | B | FER ref | FER GPU (pooled) | GPU 99% band at B | BER ref | BER GPU (pooled) | GPU 99% band at B |")
    print("|---|---|---|---|---|---|---|---|")
    for r in rows:
        print(f"| {r['snr_db']:.1f} | {r['B']} | {r['fer_ref']:.4f} | {r['fer_gpu']:.4f} | "
              f"[{r['fer_lo']:.4f}, {r['fer_hi']:.4f}] | {r['ber_ref']:.2e} | {r['ber_gpu']:.2e} | "
              f"[{r['ber_lo']:.2e}, {r['ber_hi']:.2e}] |")
    print(json.dumps(rows))


if __name__ == "__main__":
    main()
