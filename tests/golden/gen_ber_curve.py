#!/usr/bin/env python3
"""Reference BER/FER curve for the north-star's "BER curve overlaying the CPU
reference at Eb/N0 1.0-3.0 dB" (BASELINE.json).

Runs ONLY in the build container, where the reference CLI runs
(no permission denial).  It starts the reference's own
`main.py` (python_ldpc_app/main.py:451-) as a child process, once per SNR
point, with its own time-seeded channel and generator (channel.py:38-81,
data_buffer.py:47-82, generator.py:7-9), SPA, max 50 iterations, --ber --fer,
and records the per-point counters from its --output-json file
(results.py:9-117).  Only those counters are committed
(tests/golden/ber_curve_wimax_576_0.5.json); tests/test_gpu_mc.py checks that
the GPU Monte-Carlo sweep at the same points lies inside the binomial
confidence interval of the reference's FER (and the BER ratio band).

Usage:  python tests/golden/gen_ber_curve.py [--code wimax_576_0.5] [--threads 6]
                                            [--points 1.0:96,1.5:128,...]
The north-star code (round 2): --code wimax_2304_0.5 --threads 4
--points 3.0:64,1.0:8,2.0:16 (a 2304 frame-iteration costs ~25 s of one core
in the reference, so the frame counts are small; the GPU test compares the
reference's counts with the distribution of the GPU's at the same count).
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

REF_APP = "/root/reference/python_ldpc_app"
REF_DB = "/root/reference/Channel_Codes_Database"
HERE = os.path.dirname(os.path.abspath(__file__))
T = 50
DEFAULT_POINTS = "1.0:96,1.5:128,2.0:192,2.5:256,3.0:384"


def run_point(alist, snr, blocks, threads, tmp):
    out = os.path.join(tmp, f"snr_{snr}.json")
    cmd = [sys.executable, os.path.join(REF_APP, "main.py"), "--matrix", alist, "--blocks", str(blocks),
           "--iterations", str(T), "--decoder", "sumproduct", "--initial-snr", str(snr),
           "--end-snr", str(snr), "--step-snr", "0.5", "--ber", "--fer", "--threads", str(threads),
           "--output-json", out]
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    t0 = time.time()
    subprocess.run(cmd, check=True, cwd=tmp, env=env, stdout=subprocess.DEVNULL)
    res = json.load(open(out))
    pts = res["snr_points"]
    assert len(pts) == 1, pts
    p = pts[0]
    k = res["config"]["k"]
    err_bits = round(p["ber"] * k * blocks)
    return {"snr_db": snr, "blocks": blocks, "failed": p["failed_blocks"], "err_bits": err_bits,
            "fer": p["fer"], "ber": p["ber"], "avg_conv": p["avg_convergence_iterations"],
            "wall_s": round(time.time() - t0, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--code", default="wimax_576_0.5")
    ap.add_argument("--threads", type=int, default=6)
    ap.add_argument("--points", default=DEFAULT_POINTS)
    ap.add_argument("--out", default=None)
    ap.add_argument("--append", action="store_true",
                    help="run points already in the file again and add the counts")
    a = ap.parse_args()
    CODE = a.code
    alist = os.path.join(REF_DB, "Wimax LDPC Codes", CODE + ".alist.txt")
    a.out = a.out or os.path.join(HERE, f"ber_curve_{CODE}.json")
    points = [(float(s), int(b)) for s, b in (x.split(":") for x in a.points.split(","))]
    doc = {"code": CODE, "max_iter": T, "decoder": "sumproduct", "channel_mode": 1, "speed": 1.0,
           "source": "reference python_ldpc_app/main.py run in the build container (time-seeded RNG)",
           "generator": "tests/golden/gen_ber_curve.py", "points": []}
    if os.path.exists(a.out):  # resume: keep points already measured
        doc = json.load(open(a.out))
    done = {p["snr_db"] for p in doc["points"]}
    with tempfile.TemporaryDirectory() as tmp:
        for snr, blocks in points:
            if snr in done and not a.append:
                continue
            r = run_point(alist, snr, blocks, a.threads, tmp)
            r["threads"] = a.threads
            print(json.dumps(r), flush=True)
            if snr in done:
                # --append: another independent run of the reference at the same point
                # (its RNG is time-seeded); the counts of the runs add up
                p = next(q for q in doc["points"] if q["snr_db"] == snr)
                runs = p.pop("runs", None) or [dict(p)]
                runs.append(r)
                p["blocks"] = sum(x["blocks"] for x in runs)
                p["failed"] = sum(x["failed"] for x in runs)
                p["err_bits"] = sum(x["err_bits"] for x in runs)
                p["fer"] = p["failed"] / p["blocks"]
                p["ber"] = sum(x["ber"] * x["blocks"] for x in runs) / p["blocks"]
                p["wall_s"] = round(sum(x["wall_s"] for x in runs), 1)
                p["runs"] = runs
                json.dump(doc, open(a.out, "w"), indent=1)
                continue
            doc["points"].append(r)
            doc["points"].sort(key=lambda p: p["snr_db"])
            json.dump(doc, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
