#!/usr/bin/env python3
"""CPU-baseline calibration: the C oracle (bench.py's cpu_baseline, kind
"port") against the reference's own main.py on the same code, SNR, iteration
cap and number of cores, in the build container.

The reference side comes from tests/golden/ber_curve_<code>.json (written by
tests/golden/gen_ber_curve.py, which runs python_ldpc_app/main.py --threads T
and records its wall clock).  Its frame-iterations are reconstructed from the
recorded counters: failed frames ran max_iter iterations, converged frames
avg_conv + 1.  The oracle decodes freshly generated frames of the same code
and SNR with the same thread count (OpenMP over frames) and reports the same
quantity.  The ratio says how much faster the port is than the reference per
core, so bench.py's cpu_baseline (the port on the GPU box's cores) can be read
as a reference-equivalent number.

usage: python tools/calibrate_cpu.py [--code wimax_2304_0.5] [--frames 64]
writes profiles/r2_cpu_calibration/calibration.json
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "ldpc-simulator_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

EDD_BUILD_S = 55.1  # reference EncoderDecoderData for wimax_2304_0.5, gen_golden.py log (one core)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--code", default="wimax_2304_0.5")
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r2_cpu_calibration", "calibration.json"))
    a = ap.parse_args()
    import numpy as np
    import oracle
    from conftest import hstd_for

    ref = json.load(open(os.path.join(ROOT, "tests", "golden", f"ber_curve_{a.code}.json")))
    T = int(ref["max_iter"])
    H = hstd_for(a.code)
    rows = []
    for p in ref["points"]:
        thr = int(p.get("threads", 6))
        conv_frames = p["blocks"] - p["failed"]
        ref_iters = p["failed"] * T + conv_frames * (p["avg_conv"] + 1.0)
        ref_s = max(p["wall_s"] - EDD_BUILD_S, 1e-9)  # main.py builds H_std once before the loop
        sigma = oracle.sigma_for_snr(p["snr_db"])
        _, _, llr = oracle.generate_frames(H, 20260213, 0, sigma, 0, a.frames)
        t0 = time.perf_counter()
        r = oracle.spa_decode(H, llr, T, want_L=False, threads=thr)
        dt = time.perf_counter() - t0
        o_iters = int(np.asarray(r["iters"]).sum())
        rows.append({
            "snr_db": p["snr_db"], "threads": thr,
            "reference": {"frames": p["blocks"], "frame_iterations": ref_iters, "seconds": ref_s,
                          "frame_iterations_per_s": ref_iters / ref_s, "codewords_per_s": p["blocks"] / ref_s},
            "oracle": {"frames": a.frames, "frame_iterations": o_iters, "seconds": dt,
                       "frame_iterations_per_s": o_iters / dt, "codewords_per_s": a.frames / dt},
            "oracle_over_reference_per_iteration": (o_iters / dt) / (ref_iters / ref_s),
        })
        print(json.dumps(rows[-1]), flush=True)
    doc = {"code": a.code, "max_iter": T, "host": "build container (8 CPUs)",
           "reference_source": f"tests/golden/ber_curve_{a.code}.json (python_ldpc_app/main.py --threads T)",
           "oracle": "oracle/spa_oracle.c -O2, OpenMP over frames, same thread count",
           "edd_build_seconds_subtracted": EDD_BUILD_S, "points": rows}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(doc, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
