#!/usr/bin/env python3
"""Headline benchmark: decoded codewords/s (+ info-bits/s) of the on-device
Monte-Carlo step on MI355X, BASELINE.json configs[2] (the north-star code):

    WiMAX n=2304 rate-1/2 (wimax_2304_0.5), SPA fp64, max 50 iterations with
    the reference's early-termination syndrome, reference SNR axis 1.0 dB
    (speed 1.0).  The config's 262,144-frame batch is run as 32,768-frame
    steps with the global frame index continuing (8 steps cover the batch).

A step = one pass of the hot path over one batch: generate 32,768 synthetic
frames on the GPU (info bits -> [u, A.u] -> BPSK -> AWGN -> LLR), decode them
(up to 50 iterations with early termination) and reduce the main.py counters
on the device.  With N GPUs (one process per GPU, launched by
torch.distributed.run) every rank decodes its own disjoint frame range and the
counters are summed with ONE all-reduce over RCCL (weak scaling).  After the
timed region, one step each at --extra-snr points (default 2.0 and 3.0 dB) is
timed and reported under "snr_points" (scope "step"), then --point-snr (default
3.0 dB) as ONE whole config-3 point of 262,144 frames per GPU streamed in one
run (scope "point": the streaming tail is paid once per point, as main.py pays
it), a few steps of the physical mode (the
north-star's absolute cw/s target, NOT the reference's arithmetic) under
"physical" at the headline's SNR and at a waterfall point, and BASELINE
config 4 under "config4": wimax_2304_0.75A over main.py's 1.0:0.5:4.0 dB grid,
32,768 frames per GPU per point (one GPU's shard of 262,144), each point one
streaming run of the 8-frame sub-tile decoder, plus one static tile8 step.

Launch: under torch.distributed.run (RANK / WORLD_SIZE set) every process is
one rank.  `bench.py --gpus N` (N > 1) with no launcher around it starts its
own N rank processes (self_launch: fresh children, before anything touches
HIP) -- as the reference's main.py starts its own worker pool
(python_ldpc_app/main.py:248-291).  `n_gpus` in the JSON line is the number of
ranks that answered on the communicator (`ranks_seen`), never the flag.

Output: ONE JSON line on rank 0 (contract in the task statement), with
`roofline` for the whole decode (algorithmic bytes, SURVEY.md section 8d, over
the decode kernels' HIP-event time on the decoder's stream) and `cpu_baseline`
(the C oracle, OpenMP over all usable host cores, bounded sample).
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ldpc-simulator_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
SEED = 20260213
METRIC = "decoded codewords/s + info-bits/s at fixed (N, rate, max_iter, Eb/N0)"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--code", default="wimax_2304_0.5")
    ap.add_argument("--frames", type=int, default=32768, help="frames per GPU per step")
    ap.add_argument("--chunk", type=int, default=0,
                    help="decoder slots (frames resident at once); 0 = whole batch, capped by an HBM budget "
                         "(Decoder.fit_slots, --hbm-budget-gb)")
    ap.add_argument("--hbm-budget-gb", type=float, default=220.0,
                    help="HBM the decoder workspace may take (of 288 GB per MI355X)")
    ap.add_argument("--schedule", choices=("auto", "stream", "static"), default="auto",
                    help="stream: a slot takes the next frame as soon as its frame stops; static: chunks decoded "
                         "to completion (same frames, same counters); auto: static where the tile-resident "
                         "decoder applies (one launch per chunk, tiles exit on their own), else stream")
    ap.add_argument("--split", action="store_true",
                    help="parity mode: per-iteration CN/VN launches even where the tile-resident decoder applies")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--snr", type=float, default=1.0, help="reference SNR axis (dB), speed=1")
    ap.add_argument("--extra-snr", default="2.0,3.0",
                    help="comma-separated SNR points timed for one step each after the headline ('' = none)")
    ap.add_argument("--point-snr", default="3.0",
                    help="comma-separated SNR points streamed as ONE whole point of --point-frames frames per GPU "
                         "(config 3's per-SNR batch; the streaming tail is paid once per point, as in main.py's "
                         "per-point loop) and reported under 'snr_points' with scope 'point' ('' = none)")
    ap.add_argument("--point-frames", type=int, default=262144, help="frames per GPU of a whole --point-snr point")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline sample budget (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every usable host core (usable_cores())")
    ap.add_argument("--mode", choices=("parity", "physical"), default="parity",
                    help="parity: the reference's fp64 decoder on H_std (headline); physical: "
                         "SURVEY §8 f4, standard SPA on the sparse graph, fp32, LDS-resident")
    ap.add_argument("--phys-hbm", action="store_true",
                    help="physical mode: HBM-resident state even when a frame fits in LDS")
    ap.add_argument("--phys-steps", type=int, default=4,
                    help="parity mode: timed physical-mode steps reported under 'physical' after the "
                         "headline (0 = none); not the reference's arithmetic (SURVEY 8 f4)")
    ap.add_argument("--phys-waterfall-snr", type=float, default=-2.5,
                    help="parity mode: a second physical-mode point in the waterfall, where the decoder "
                         "iterates (reported under physical.waterfall; NaN = none)")
    ap.add_argument("--phys-frames", type=int, default=262144,
                    help="frames per physical-mode step (config 3's batch; 65,536 measured 2.7 %% slower: host syncs)")
    ap.add_argument("--config4-snr", default="1.0:0.5:4.0",
                    help="parity mode: BASELINE config 4's Eb/N0 sweep (start:step:end, main.py's grid) on "
                         "--config4-code, reported under 'config4' ('' = none)")
    ap.add_argument("--config4-code", default="wimax_2304_0.75A")
    ap.add_argument("--config4-frames", type=int, default=32768,
                    help="frames per GPU per config-4 point (one GPU's shard of 262,144 over 8 GPUs)")
    ap.add_argument("--config4-slots", type=int, default=2048,
                    help="streaming slots of the config-4 decoder (256 CUs x one 8-frame tile8 workgroup)")
    ap.add_argument("--config2", type=int, default=1,
                    help="parity mode: BASELINE config 2 (wimax_576_0.5, T=50, 65,536 frames, 0 dB) timed for "
                         "--config2-steps steps under 'config2' (0 = none)")
    ap.add_argument("--config2-steps", type=int, default=3)
    ap.add_argument("--config5", type=int, default=1,
                    help="parity mode: BASELINE config 5 (DVB-S2 n=64800 r1/2 profile, physical mode only: its "
                         "H_std would have ~5e8 edges) under 'config5' (0 = none)")
    ap.add_argument("--config5-frames", type=int, default=8192, help="config-5 frames per GPU per step")
    ap.add_argument("--config5-waterfall-snr", type=float, default=-2.5,
                    help="a second config-5 point in the waterfall, where the 50-iteration decoder iterates "
                         "(~30 average iterations at -2.5 dB; NaN = none)")
    ap.add_argument("--dropin-calls", type=int, default=20,
                    help="parity mode: one-frame decode() calls timed under 'dropin' (main.py's call pattern; 0 = none)")
    ap.add_argument("--stub", action="store_true",
                    help="launcher rehearsal without a GPU: every rank only joins a gloo group and "
                         "counts the ranks (tests/test_bench_launch.py); also LDPC_BENCH_STUB=1")
    return ap.parse_args()


def self_launch(args, argv):
    """`bench.py --gpus N` (N > 1) with no launcher around it: start N fresh
    child processes of this script, rank r on GPU r, each with RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT and one rendezvous key
    for the whole launch (LDPC_RDV_KEY, ldpc_amd.comm).  Runs before anything
    imports ldpc_amd or touches HIP, and starts the children with subprocess
    (never exec).  Rank 0's stdout (the JSON line) is ours; the other ranks'
    stdout is discarded.  If a rank fails, the others are stopped and the
    launch exits non-zero.  -> exit status."""
    import signal
    import socket
    import subprocess
    import uuid
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    key = uuid.uuid4().hex
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   LDPC_RDV_KEY=key)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                print(f"bench.py: rank {procs.index(p)} exited with {rc}; stopping the other ranks",
                      file=sys.stderr)
                for q in live:  # the processes this launcher started, by their own handles
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.05)
    return status


def stub_rank(args, world, rank):
    """--stub: the launcher's contract without a GPU -- join a gloo group of
    WORLD_SIZE ranks, count them, rank 0 prints the JSON line."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://{os.environ.get('MASTER_ADDR', '127.0.0.1')}:"
                                                f"{os.environ.get('MASTER_PORT', '29500')}",
                            rank=rank, world_size=world)
    t = torch.ones(1, dtype=torch.int64)
    dist.all_reduce(t)
    seen = int(t.item())
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "stub": True, "n_gpus": seen, "ranks_seen": seen,
                          "world_size": world, "gpus_flag": args.gpus,
                          "rdv_key_set": bool(os.environ.get("LDPC_RDV_KEY"))}), flush=True)
    dist.destroy_process_group()


class RcclDist:
    """The N>1 exchange through the C ABI (ldpc_amd.comm: RCCL over xGMI, file
    rendezvous of the unique id, no PyTorch)."""

    def __init__(self, device):
        from ldpc_amd.comm import Comm
        self.c = Comm.from_env(device)
        self.device = device

    def allreduce(self, ctr):
        return self.c.allreduce(np.asarray(ctr, np.int64))

    def max(self, x):
        return float(self.c.allreduce(np.array([x], np.float64), op="max")[0])

    def barrier(self):
        self.c.barrier()  # all ranks arrive, then hipDeviceSynchronize

    def ranks_seen(self):
        return self.c.ranks_seen()

    def close(self):
        self.c.close()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # LDPC_BENCH_FORCE_DIST=1: the N>1 code path (communicator, counter
    # all-reduce, barriers, max over ranks) with a single rank -- how the
    # driver's multi-GPU run is rehearsed on a one-GPU box
    if world > 1 or os.environ.get("LDPC_BENCH_FORCE_DIST") == "1":
        dist = RcclDist(local)
    return world, rank, local, dist


def allreduce_counters(dist, ctr, local):
    """The single all-reduce of the error counters (int64 [points x 7])."""
    return ctr if dist is None else dist.allreduce(ctr)


def barrier(dist, local):
    if dist is not None:
        dist.barrier()


def max_over_ranks(dist, x, local):
    return x if dist is None else dist.max(x)


VALU_PEAK = 256 * 4 * 2.4e9 / 2.0  # wave64 VALU instructions/s (2 cycles each per SIMD)


def committed_valu(code, kernel, snr_db):
    """VALU wave-instructions per frame-iteration of `kernel` on `code` at this
    SNR from the newest committed profile (tools/profile_phys.sh +
    summarize_phys_profile.py: profiles/<tag>/valu*.json).  The count per
    frame-iteration depends on the operating point (per-pass overheads are
    shared by fewer iterations when frames stop early), so only a profile of
    the same SNR counts."""
    pdir = os.path.join(ROOT, "profiles")
    best = (None, None)
    for d in sorted(os.listdir(pdir), key=profile_order) if os.path.isdir(pdir) else []:
        if not os.path.isdir(os.path.join(pdir, d)):
            continue
        for fn in sorted(os.listdir(os.path.join(pdir, d))):
            if not (fn.startswith("valu") and fn.endswith(".json")):
                continue
            f = os.path.join(pdir, d, fn)
            v = json.load(open(f))
            if v.get("code") == code and v.get("kernel") == kernel and \
                    abs(float(v.get("snr_db", 1e9)) - snr_db) < 1e-9:
                best = (v["valu_insts_per_frame_iteration"], os.path.relpath(f, ROOT))
    return best


def profile_order(d):
    """Chronological order of profiles/ tags r<round><letters>_...: within a
    round a..z, then aa..zz (so r2z < r2aa < r2as)."""
    import re
    mt = re.match(r"r(\d+)([a-z]*)", d)
    return (int(mt.group(1)), len(mt.group(2)), mt.group(2), d) if mt else (-1, 0, "", d)


def committed_traffic(nnz, frames, kernel="cn", snr=None):
    """HBM bytes per cn_kernel launch from the newest committed PMC pass
    (profiles/*/traffic.json, tools/profile.sh + tools/summarize_profile.py)
    for this exact workload shape (and SNR, where the file records one and
    `snr` is given), or (None, None)."""
    pdir = os.path.join(ROOT, "profiles")
    best = None
    for d in sorted(os.listdir(pdir), key=profile_order) if os.path.isdir(pdir) else []:
        if not os.path.isdir(os.path.join(pdir, d)):
            continue
        for fn in sorted(os.listdir(os.path.join(pdir, d))):
            if not (fn.startswith("traffic") and fn.endswith(".json")):
                continue
            f = os.path.join(pdir, d, fn)
            t = json.load(open(f))
            if snr is not None and "snr_db" in t and abs(float(t["snr_db"]) - snr) > 1e-9:
                continue
            if t.get("edges") == nnz and t.get("frames") == frames:
                k = t.get("kernels", {})
                cn = k.get(kernel) or (k.get("cn_kernel<false>") if kernel == "cn" else None)
                if cn:
                    best = (cn["traffic_bytes"], os.path.relpath(f, ROOT))
    return best or (None, None)


def usable_cores():
    """Host cores this process may run on: the affinity mask, capped by the
    cgroup CPU quota when one is set (a GPU box's share of a larger machine:
    os.cpu_count() there counts the whole machine).  -> (cores, affinity, quota)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            parts = open(path).read().split()
        except OSError:
            continue
        if path.endswith("cpu.max") and parts and parts[0] != "max":
            quota = int(parts[0]) / int(parts[1])
        elif path.endswith("quota_us") and parts and int(parts[0]) > 0:
            period = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            quota = int(parts[0]) / period
        break
    cores = aff if quota is None else max(1, min(aff, int(math.ceil(quota))))
    return cores, aff, quota


def cpu_baseline(H, k, args):
    """The C oracle (oracle/spa_oracle.c, OpenMP over frames) on a bounded
    sample of the same workload; frames from the oracle's restatement of the
    device frame source.  Every usable host core (usable_cores())."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    cores, aff, quota = usable_cores()
    threads = args.cpu_threads or cores
    sigma = oracle.sigma_for_snr(args.snr)
    per = max(2 * threads, 16)
    done, iters, t0 = 0, 0, time.perf_counter()
    batch = 0
    while True:
        _, _, llr = oracle.generate_frames(H, SEED, 0, sigma, batch * per, per)
        r = oracle.spa_decode(H, llr, args.iters, want_L=False, threads=threads)
        done += per
        iters += int(r["iters"].sum())
        batch += 1
        if time.perf_counter() - t0 >= args.cpu_seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "codewords/s", "cores": threads, "kind": "port",
            "sample": f"{done} frames of {args.code}, T={args.iters}, snr={args.snr} dB "
                      f"({iters} frame-iterations) in {dt:.1f} s; oracle/spa_oracle.c -O2 OpenMP, "
                      f"{threads} threads",
            "host_cpus_affinity": aff, "cgroup_cpu_quota": quota,
            "calibration": "profiles/r2_cpu_calibration/calibration.json (oracle vs the reference main.py, "
                           "same config and cores, build container)",
            "info_bits_per_s": done * k / dt}


def cpu_baseline_phys(H, k, args, ira_code):
    """Physical mode: its CPU restatement (oracle/phys_oracle.c, one frame per
    thread call, threads via ctypes which releases the GIL) on a bounded sample."""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    threads = args.cpu_threads or usable_cores()[0]
    sigma = oracle.sigma_for_snr(args.snr)
    Hp, Hgen = H

    def one(i):
        _, _, llr = oracle.generate_frames(Hgen, SEED, 0, sigma, i * 4, 4, ira=ira_code)
        return int(oracle.phys_decode(Hp, llr, args.iters)["iters"].sum())

    done, iters, t0, i = 0, 0, time.perf_counter(), 0
    with ThreadPoolExecutor(threads) as ex:
        while time.perf_counter() - t0 < args.cpu_seconds:
            iters += sum(ex.map(one, range(i, i + threads)))
            done += 4 * threads
            i += threads
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "codewords/s", "cores": threads, "kind": "port",
            "sample": f"{done} frames of {args.code} (physical mode), T={args.iters}, snr={args.snr} dB "
                      f"({iters} frame-iterations) in {dt:.1f} s; oracle/phys_oracle.c -O2, {threads} threads",
            "info_bits_per_s": done * k / dt}


IRA_CODES = {"dvbs2_profile_64800_0.5": "dvbs2_profile_matrix"}


def physical_extra(args, edd, graph, local, world, rank, dist, k):
    """The north-star's absolute target (>= 1e8 cw/s on wimax_2304_0.5 at 50
    max iterations over 8 GPUs) is reachable only in physical mode (SURVEY 8d,
    8 f4): standard SPA on the sparse graph H[:, perm], sign-consistent, fp32,
    a frame's state in LDS.  NOT the reference's arithmetic (no parity): timed
    here after the parity headline, outside its timed region, over the same
    code, max_iter and on-device frame source, on frame indices disjoint from
    the headline's -- at the headline's SNR (1 dB on the reference axis, where
    the reference channel's noise std sigma^2 makes frames converge in ~1
    iteration) and at a waterfall point (--phys-waterfall-snr, -2.5 dB: ~35
    iterations, FER ~0.4) where the decoder actually iterates.  Roofline = VALU
    issue (the state never leaves LDS): committed PMC VALU instructions per
    frame-iteration of the same kernel, code and SNR x this run's
    frame-iterations / the kernel's HIP-event time."""
    from ldpc_amd import _lib
    from ldpc_amd.device import Decoder, Graph
    pg = Graph(edd.physical_matrix(), device=local)
    B = args.phys_frames
    pdec = Decoder(graph, B)  # frame source = H_std; E is never allocated in physical mode
    name = _lib.lib().ldpc_phys_kernel_name(pg.handle, 0).decode()

    def point(snr, base):
        sig = 1.0 / math.sqrt(2.0 * 1.0 * (10.0 ** (snr * 0.1)))
        pdec.phys_mc_run(pg, SEED, [sig], B, base + rank * B, args.iters)  # untimed warm-up
        barrier(dist, local)
        pdec.profile_read()
        pdec.profile(True)
        barrier(dist, local)
        t0 = time.perf_counter()
        loc = np.zeros((1, 7), np.int64)
        tot = np.zeros((1, 7), np.int64)
        for s in range(args.phys_steps):
            c = pdec.phys_mc_run(pg, SEED, [sig], B, base + ((s + 1) * world + rank) * B, args.iters)
            loc += c
            tot += allreduce_counters(dist, c, local)
        barrier(dist, local)
        dt = max_over_ranks(dist, time.perf_counter() - t0, local)
        pdec.profile(False)
        pms, pl = pdec.profile_read()["phys"]
        frames = int(tot[0, 0])
        out = {"value": frames / dt, "unit": "codewords/s", "per_gpu": frames / dt / world, "n_gpus": world,
               "steps": args.phys_steps, "frames_per_gpu_step": B, "ms_per_step": dt / args.phys_steps * 1e3,
               "info_bits_per_s": frames * k / dt, "dtype": "f32", "snr_db": snr, "max_iter": args.iters,
               "edges_H_phys": int(pg.nnz), "fer": int(tot[0, 1]) / max(frames, 1),
               "ber": int(tot[0, 2]) / (k * max(frames, 1)), "avg_iters": int(tot[0, 6]) / max(frames, 1),
               "kernel": name, "kernel_ms": pms, "launches": pl}
        vi, vsrc = committed_valu(args.code, name, snr)
        if vi and pms:
            ach = vi * int(loc[0, 6]) / (pms / 1e3)
            out["roofline"] = {"bound": "valu", "achieved": ach, "peak": VALU_PEAK, "unit": "VALU wave-instr/s",
                               "frac": ach / VALU_PEAK, "valu_insts_per_frame_iteration": vi, "valu_source": vsrc,
                               "peak_model": "256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 fp32 VALU "
                                             "instruction (MI355X_MICROARCH.md)"}
        return out

    out = {"what": "physical mode (SURVEY 8 f4): standard SPA on the sparse H[:,perm], sign-consistent, fp32, "
                   "state in LDS -- NOT the reference's arithmetic, no parity with spa_decoder.py; timed after "
                   "and outside the parity headline",
           "north_star_target_cw_s_8gpu": 1e8}
    out.update(point(args.snr, 1 << 42))  # far from the parity steps' frame ranges
    if not math.isnan(args.phys_waterfall_snr):
        out["waterfall"] = point(args.phys_waterfall_snr, (1 << 42) + (1 << 38))
    pdec.close()
    return out


def snr_grid(spec):
    """'start:step:end' -> main.py's SNR grid (ldpc_amd.montecarlo.snr_grid,
    main.py:193,206-209), or a comma list."""
    if ":" not in spec:
        return [float(v) for v in spec.split(",") if v.strip()]
    from ldpc_amd.montecarlo import snr_grid as grid
    a, st, b = (float(v) for v in spec.split(":"))
    return [float(x) for x in grid(a, b, st)]


def config4_extra(args, local, world, rank, dist):
    """BASELINE config 4: wimax_2304_0.75A, Eb/N0 sweep 1.0..4.0 dB, T=50 with
    early termination, frames sharded over the GPUs (this rank: its own
    --config4-frames per point, disjoint global frame ranges) with the counter
    all-reduce per point.  Each point is ONE streaming mc_run call: the
    8-frame sub-tile decoder tile8_stream_kernel (per-slot refill by gen_slots)
    with the hand-off of its last running frames to the column-parallel split
    tail.  Per point: cw/s, the main.py counters, and the whole decode's
    algorithmic bytes (8 n + 16 B x edges x iterations + ceil(n/8) +
    8 per frame) over the decode kernels' HIP-event time (stream kernel + tail
    CN/VN + refills).  Then one static 32,768-frame step at 1 dB through
    tile8_kernel (every frame runs 50 iterations there), the r3/4 decoder's
    fused-kernel roofline like the headline's."""
    import ldpc_amd
    from ldpc_amd import _lib
    from ldpc_amd.device import Decoder, Graph
    edd = ldpc_amd.load_committed_code(args.config4_code)
    H = edd._h_std
    n, k, nnz = edd._n, edd._k, H.nnz
    g = Graph(H, device=local)
    F = args.config4_frames
    dec = Decoder(g, min(args.config4_slots, F))
    sig = lambda x: 1.0 / math.sqrt(2.0 * 1.0 * (10.0 ** (x * 0.1)))  # noqa: E731  channel.py:113
    base = 1 << 43  # far from every other key's frame ranges
    dec.mc_run(SEED, [sig(2.5)], 256, base - 4096, args.iters)  # untimed warm-up (workspace, first launches)
    pts, tot_f, tot_t, tot_b, tot_ms = [], 0, 0.0, 0.0, 0.0
    kinds = ("tile", "cn", "vn", "vn_cols", "generate")
    for i, x in enumerate(snr_grid(args.config4_snr)):
        barrier(dist, local)
        dec.profile_read()
        dec.profile(True)
        t1 = time.perf_counter()
        loc = dec.mc_run(SEED, [sig(x)], F, base + (i * world + rank) * F, args.iters)
        c = allreduce_counters(dist, loc, local)
        barrier(dist, local)
        dt = max_over_ranks(dist, time.perf_counter() - t1, local)
        dec.profile(False)
        prof = dec.profile_read()
        f = int(c[0, 0])
        ms = sum(prof[kk][0] for kk in kinds)
        byts = F * (8 * n + math.ceil(n / 8) + 8) + 16.0 * nnz * int(loc[0, 6])  # this rank
        pts.append({"snr_db": x, "value": f / dt, "unit": "codewords/s", "info_bits_per_s": f * k / dt,
                    "ms": dt * 1e3, "frames": f, "avg_iters": int(c[0, 6]) / max(f, 1),
                    "fer": int(c[0, 1]) / max(f, 1), "ber": int(c[0, 2]) / (k * max(f, 1)),
                    "decode_ms": ms, "stream_kernel_ms": prof["tile"][0],
                    "tail_ms": prof["cn"][0] + prof["vn"][0] + prof["vn_cols"][0],
                    "roofline_frac": byts / (ms / 1e3) / 1e9 / HBM_PEAK_GBS if ms else None})
        tot_f += f
        tot_t += dt
        tot_b += byts
        tot_ms += ms
    dec.close()
    out = {"what": "BASELINE config 4: Eb/N0 sweep, one streaming mc_run per point (tile8_stream_kernel + "
                   "column-parallel tail), counters all-reduced per point",
           "code": args.config4_code, "n": n, "k": k, "edges_H_std": nnz, "max_iter": args.iters,
           "frames_per_gpu_per_point": F, "slots": min(args.config4_slots, F), "n_gpus": world,
           "kernel": _lib.lib().ldpc_tile_kernel_name(g.handle).decode().replace("_kernel", "_stream_kernel"),
           "value": tot_f / tot_t, "unit": "codewords/s", "info_bits_per_s": tot_f * k / tot_t,
           "points": pts,
           "roofline": {"bound": "hbm", "achieved": tot_b / (tot_ms / 1e3) / 1e9, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": tot_b / (tot_ms / 1e3) / 1e9 / HBM_PEAK_GBS,
                        "bytes_model": "whole sweep, this rank: per frame 8 n + 16 B x H_std edges x iterations "
                                       "executed + ceil(n/8) + 8 (SURVEY 8d), over the decode kernels' HIP-event "
                                       "time (stream kernel + tail + refills)"}}
    tr, tsrc = committed_traffic(nnz, min(args.config4_slots, F), "tile8_stream")
    if tr is not None:
        out["roofline"]["traffic"] = tr
        out["roofline"]["traffic_source"] = tsrc
    # the fused static decoder (tile8_kernel) at 1 dB: one 32,768-frame launch, all 50 iterations
    sdec = Decoder(g, F)
    sdec.mc_run(SEED, [sig(1.0)], 2048, base - 2 * F - 4096, args.iters, static=True)  # warm-up (tile8 from 17 tiles)
    barrier(dist, local)
    sdec.profile_read()
    sdec.profile(True)
    t1 = time.perf_counter()
    loc = sdec.mc_run(SEED, [sig(1.0)], F, base + (1 << 40) + rank * F, args.iters, static=True)
    c = allreduce_counters(dist, loc, local)
    barrier(dist, local)
    dt = max_over_ranks(dist, time.perf_counter() - t1, local)
    sdec.profile(False)
    prof = sdec.profile_read()
    sdec.close()
    tms, tl = prof["tile"]
    byts = F * (8 * n + math.ceil(n / 8) + 8) + 16.0 * nnz * int(loc[0, 6])
    st = {"snr_db": 1.0, "schedule": "static", "frames": int(c[0, 0]), "value": int(c[0, 0]) / dt,
          "unit": "codewords/s", "avg_iters": int(c[0, 6]) / max(int(c[0, 0]), 1),
          "kernel": _lib.lib().ldpc_tile_kernel_name(g.handle).decode(), "launches": tl,
          "avg_launch_ms": tms / max(tl, 1)}
    if tl:
        st["roofline"] = {"bound": "hbm", "achieved": byts / (tms / 1e3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": byts / (tms / 1e3) / 1e9 / HBM_PEAK_GBS, "bytes_per_launch": byts / tl}
        tr, tsrc = committed_traffic(nnz, F, "tile")
        st["roofline"]["traffic"], st["roofline"]["traffic_source"] = tr, tsrc
    out["static_1dB"] = st
    return out


def config2_extra(args, local, world, rank, dist):
    """BASELINE config 2: wimax_576_0.5, SPA fp64, T=50 with early termination,
    65,536 frames per GPU per step at the reference axis' 0 dB (FER 1.0 in the
    reference: every frame runs 50 iterations), static schedule -> one
    tile_kernel launch per step (64 frames per workgroup, CN + VN fused)."""
    import ldpc_amd
    from ldpc_amd import _lib
    from ldpc_amd.device import Decoder, Graph
    edd = ldpc_amd.load_committed_code("wimax_576_0.5")
    H = edd._h_std
    n, k, nnz = edd._n, edd._k, H.nnz
    g = Graph(H, device=local)
    F = 65536
    dec = Decoder(g, F)
    sig = 1.0 / math.sqrt(2.0)  # 0 dB, speed 1 (channel.py:113)
    base = 1 << 44
    dec.mc_run(SEED, [sig], F, base - F, args.iters, static=True)  # warm-up
    barrier(dist, local)
    dec.profile_read()
    dec.profile(True)
    t1 = time.perf_counter()
    loc = np.zeros((1, 7), np.int64)
    tot = np.zeros((1, 7), np.int64)
    for st in range(args.config2_steps):
        c = dec.mc_run(SEED, [sig], F, base + (st * world + rank) * F, args.iters, static=True)
        loc += c
        tot += allreduce_counters(dist, c, local)
    barrier(dist, local)
    dt = max_over_ranks(dist, time.perf_counter() - t1, local)
    dec.profile(False)
    tms, tl = dec.profile_read()["tile"]
    dec.close()
    f = int(tot[0, 0])
    byts = F * args.config2_steps * (8 * n + math.ceil(n / 8) + 8) + 16.0 * nnz * int(loc[0, 6])
    out = {"what": "BASELINE config 2: wimax_576_0.5 SPA fp64, T=50 + early termination, 0 dB (FER 1.0 in the "
                   "reference), 65,536 frames per GPU per step, static schedule",
           "code": "wimax_576_0.5", "n": n, "k": k, "edges_H_std": nnz, "snr_db": 0.0, "max_iter": args.iters,
           "frames_per_gpu_step": F, "steps": args.config2_steps, "n_gpus": world,
           "value": f / dt, "unit": "codewords/s", "info_bits_per_s": f * k / dt,
           "ms_per_step": dt / args.config2_steps * 1e3, "avg_iters": int(tot[0, 6]) / max(f, 1),
           "fer": int(tot[0, 1]) / max(f, 1),
           "kernel": _lib.lib().ldpc_tile_kernel_name(g.handle).decode(), "launches": tl}
    if tl:
        tr, tsrc = committed_traffic(nnz, F, "tile")
        out["roofline"] = {"bound": "hbm", "achieved": byts / (tms / 1e3) / 1e9, "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": byts / (tms / 1e3) / 1e9 / HBM_PEAK_GBS,
                           "avg_launch_ms": tms / tl, "bytes_per_launch": byts / tl,
                           "traffic": tr, "traffic_source": tsrc,
                           "bytes_model": "per frame 8 n + 16 B x H_std edges x iterations + ceil(n/8) + 8 "
                                          "(SURVEY 8d), CN and VN fused"}
    return out


def config5_extra(args, local, world, rank, dist):
    """BASELINE config 5: DVB-S2 n=64800 rate-1/2 at 50 max iterations, 8,192
    frames -- in physical mode only (its H_std = [A | I] would
    have ~5e8 edges).  The code has DVB-S2's exact rate-1/2 normal-frame
    structure and degree profile with a SEEDED address table (the ETSI table
    is not available offline: ldpc_amd/ira.py), so this is a stress test of
    the long irregular code's decoder, with no parity to the reference.  State
    in HBM (phys_cn_tile / phys_vn_tile), on-device IRA encoder.  Two points:
    the headline's SNR (1 dB on the reference axis: ~2 iterations) and the
    waterfall (--config5-waterfall-snr, -2.5 dB: ~30 of the 50 iterations,
    the long-block stress BASELINE names), each with the CN kernel's roofline
    and its committed PMC traffic (tools/profile_phys.sh on config 5)."""
    from ldpc_amd import ira
    from ldpc_amd.device import Decoder, Graph
    H = ira.dvbs2_profile_matrix()
    m, n = H.shape
    k = n - m
    g = Graph(H, device=local)
    F = args.config5_frames
    dec = Decoder(g, F)

    def point(snr, base):
        sig = 1.0 / math.sqrt(2.0 * (10.0 ** (snr * 0.1)))
        dec.phys_mc_run(g, SEED, [sig], F, base - F, args.iters)  # warm-up
        barrier(dist, local)
        dec.profile_read()
        dec.profile(True)
        t1 = time.perf_counter()
        loc = np.zeros((1, 7), np.int64)
        tot = np.zeros((1, 7), np.int64)
        steps = 2
        for st in range(steps):
            c = dec.phys_mc_run(g, SEED, [sig], F, base + (st * world + rank) * F, args.iters)
            loc += c
            tot += allreduce_counters(dist, c, local)
        barrier(dist, local)
        dt = max_over_ranks(dist, time.perf_counter() - t1, local)
        dec.profile(False)
        prof = dec.profile_read()
        cms, cl = prof["phys_cn"]
        f = int(tot[0, 0])
        out = {"snr_db": snr, "max_iter": args.iters, "frames_per_gpu_step": F, "steps": steps, "n_gpus": world,
               "value": f / dt, "unit": "codewords/s", "info_bits_per_s": f * k / dt,
               "ms_per_step": dt / steps * 1e3, "avg_iters": int(tot[0, 6]) / max(f, 1),
               "fer": int(tot[0, 1]) / max(f, 1), "dtype": "f32"}
        if cl:
            cn_bytes = 12.0 * H.nnz * int(loc[0, 6])
            tr, tsrc = committed_traffic(int(H.nnz), F, "phys_cn", snr)
            # compaction makes launch shapes differ between runs: compare per frame-iteration
            tfi = None
            if tsrc:
                tj = json.load(open(os.path.join(ROOT, tsrc)))
                tfi = tj.get("traffic_bytes_per_frame_iteration")
            out["roofline"] = {"bound": "hbm", "kernel": "phys_cn_tile_kernel", "launches": cl,
                               "achieved": cn_bytes / (cms / 1e3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": cn_bytes / (cms / 1e3) / 1e9 / HBM_PEAK_GBS,
                               "traffic": tr, "traffic_source": tsrc, "bytes_per_launch": cn_bytes / cl,
                               "bytes_per_frame_iteration": 12.0 * H.nnz,
                               "traffic_per_frame_iteration": tfi,
                               "traffic_ratio": tfi / (12.0 * H.nnz) if tfi else None,
                               "bytes_model": "12 B x H edges x frame-iterations (L[col] gather + E_old read + "
                                              "E_new write, fp32), over the CN launches' HIP-event time; traffic = "
                                              "committed PMC bytes per CN launch at this SNR; "
                                              "traffic_per_frame_iteration = those PMC bytes over the profiled "
                                              "run's frame-iterations, vs bytes_per_frame_iteration (the model)"}
        return out

    out = {"what": "BASELINE config 5: DVB-S2 n=64800 r1/2 profile (seeded address table), physical mode "
                   "(fp32, sparse graph, state in HBM) -- no reference parity",
           "code": "dvbs2_profile_64800_0.5", "n": n, "k": k, "edges_H": int(H.nnz)}
    out.update(point(args.snr, 1 << 45))
    if not math.isnan(args.config5_waterfall_snr):
        out["waterfall"] = point(args.config5_waterfall_snr, (1 << 45) + (1 << 40))
    dec.close()
    return out


def dropin_extra(args, graph, n):
    """main.py's call pattern through the drop-in SPA_Decoder: decode() of ONE
    frame per call (python_ldpc_app/main.py:124,312; 64 slots, as
    ldpc_amd.SPA_Decoder), which runs the few-frame edge path.  Synthetic
    frames: the all-zero codeword through the reference channel model (bit 0 ->
    -1, noise std sigma^2, LLR 2y/sigma^2: channel.py:49,68-80), host numpy RNG;
    each call uploads the frame and reads z / conv / status back, as decode()
    does.  Timed after everything else."""
    from ldpc_amd.device import Decoder
    d = Decoder(graph, 64)
    sg = 1.0 / math.sqrt(2.0 * 1.0 * (10.0 ** (args.snr * 0.1)))
    s2 = sg * sg
    rng = np.random.default_rng(SEED)
    llr = 2.0 * (-1.0 + s2 * rng.standard_normal((args.dropin_calls + 1, n))) / s2
    d.decode(llr[:1], args.iters)  # warm-up (workspace, first launches)
    iters = 0
    t0 = time.perf_counter()
    for i in range(1, args.dropin_calls + 1):
        iters += int(d.decode(llr[i:i + 1], args.iters).iters[0])
    dt = time.perf_counter() - t0
    d.close()
    return {"what": "drop-in decode(): one frame per call, main.py's loop (few-frame edge path)",
            "frames_per_call": 1, "calls": args.dropin_calls, "ms_per_call": dt / args.dropin_calls * 1e3,
            "value": args.dropin_calls / dt, "unit": "codewords/s", "avg_iters": iters / args.dropin_calls,
            "max_iter": args.iters, "snr_db": args.snr, "data": "all-zero codeword, reference channel model"}


def main():
    args = parse()
    launched = "WORLD_SIZE" in os.environ
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if not launched and args.gpus > 1:
        sys.exit(self_launch(args, sys.argv[1:]))  # nothing has touched HIP in this process
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world < args.gpus:  # fewer ranks than asked for: never report a smaller job as the N-GPU one
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if world > args.gpus:  # e.g. torchrun --nproc-per-node 8 bench.py without --gpus: the launcher's world rules
        if int(os.environ.get("RANK", "0")) == 0:
            print(f"bench.py: WORLD_SIZE={world} from the launcher, --gpus {args.gpus}: running {world} ranks",
                  file=sys.stderr)
        args.gpus = world
    if args.stub or os.environ.get("LDPC_BENCH_STUB") == "1":
        return stub_rank(args, world, int(os.environ.get("RANK", "0")))
    import ldpc_amd
    from ldpc_amd.device import Decoder, Graph

    ndev = ldpc_amd.device_count()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ndev <= 0:
        raise SystemExit("bench.py: no HIP device visible (the decoder has no CPU path)")
    if local >= ndev:
        raise SystemExit(f"bench.py: LOCAL_RANK {local} wants GPU {local} but only {ndev} are visible")
    world, rank, local, dist = dist_setup(args)
    ranks_seen = dist.ranks_seen() if dist is not None else 1
    if ranks_seen != world:
        raise SystemExit(f"bench.py: {ranks_seen} ranks answered on RCCL, WORLD_SIZE={world}")
    ira_code = args.code in IRA_CODES
    if ira_code:  # BASELINE config 5: sparse (physical) mode only, the IRA graph is its own frame source
        from ldpc_amd import ira
        if args.mode != "physical":
            raise SystemExit(f"bench.py: {args.code} runs in --mode physical only (its H_std has ~5e8 edges)")
        H = getattr(ira, IRA_CODES[args.code])()
        m, n = H.shape
        k, nnz = n - m, H.nnz
        graph = Graph(H, device=local)
        pgraph = graph
        Hphys = H
    else:
        edd = ldpc_amd.load_committed_code(args.code)
        H = edd._h_std
        n, m, k, nnz = edd._n, edd._m, edd._k, H.nnz
        graph = Graph(H, device=local)
        Hphys = edd.physical_matrix() if args.mode == "physical" else None
        pgraph = Graph(Hphys, device=local) if Hphys is not None else None
    # whole batch resident, if its state fits the HBM budget
    chunk = args.chunk or Decoder.fit_slots(graph, args.frames, budget=args.hbm_budget_gb * 1e9)
    dec = Decoder(graph, chunk)
    if args.schedule == "auto":
        from ldpc_amd import _lib
        tile_ok = pgraph is None and not args.split and _lib.lib().ldpc_tile_lds_bytes(graph.handle) > 0
        args.schedule = "static" if tile_ok else "stream"
    sigma = 1.0 / math.sqrt(2.0 * 1.0 * (10.0 ** (args.snr * 0.1)))  # channel.py:113
    B = args.frames

    local_totals = np.zeros((1, 7), np.int64)

    def step(s, record=False, sig=None, schedule=None):
        sig = sigma if sig is None else sig
        schedule = schedule or args.schedule
        frame0 = (s * world + rank) * B  # disjoint global frame ranges per rank and step
        if pgraph is not None:
            c = dec.phys_mc_run(pgraph, SEED, [sig], B, frame0, args.iters, hbm=args.phys_hbm)
        else:
            c = dec.mc_run(SEED, [sig], B, frame0, args.iters, static=schedule == "static", split=args.split)
        if record:
            local_totals[:] += c
        return allreduce_counters(dist, c, local)

    for s in range(args.warmup):
        step(s)
    barrier(dist, local)
    dec.profile_read()  # drop anything recorded so far
    dec.profile(True)
    barrier(dist, local)
    t0 = time.perf_counter()
    totals = np.zeros((1, 7), np.int64)
    for s in range(args.steps):
        totals += step(args.warmup + s, record=True)
    barrier(dist, local)
    elapsed = time.perf_counter() - t0
    dec.profile(False)
    prof = dec.profile_read()
    elapsed = max_over_ranks(dist, elapsed, local)

    # extra SNR points (one step each, after the headline's timed region), on
    # the streaming schedule: there frames stop at very different iterations,
    # so the step streams its frames through a quarter as many slots (a fresh,
    # smaller workspace) and a slot is refilled as soon as its frame stops
    snr_points = []
    extra_sched = "stream"
    extra = [v for v in args.extra_snr.split(",") if v.strip()]
    extra_slots = None
    if extra and pgraph is None:
        dec.close()
        extra_slots = max(64, (B // 4) // 64 * 64)
        dec = Decoder(graph, extra_slots)
        # untimed warm-up of the fresh workspace (lazy allocations, first launch
        # of the streaming kernel): 64 frames far outside the timed ranges
        x0 = float(extra[0])
        dec.mc_run(SEED, [1.0 / math.sqrt(2.0 * 10.0 ** (x0 * 0.1))], 64, 1 << 40, args.iters, static=False,
                   split=args.split)
    for i, x in enumerate(extra):
        x = float(x)
        sg = 1.0 / math.sqrt(2.0 * 1.0 * (10.0 ** (x * 0.1)))
        barrier(dist, local)
        t1 = time.perf_counter()
        c = step(args.warmup + args.steps + i, sig=sg, schedule=extra_sched)
        barrier(dist, local)
        dt = max_over_ranks(dist, time.perf_counter() - t1, local)
        f = int(c[0, 0])
        snr_points.append({"snr_db": x, "scope": "step", "value": f / dt, "unit": "codewords/s",
                           "info_bits_per_s": f * k / dt,
                           "ms": dt * 1e3, "frames": f, "schedule": extra_sched, "slots": extra_slots,
                           "avg_iters": int(c[0, 6]) / max(f, 1),
                           "fer": int(c[0, 1]) / max(f, 1), "ber": int(c[0, 2]) / (k * max(f, 1))})
    # whole SNR points: config 3's 262,144 frames of one point streamed through
    # the same slots in ONE mc_run (frame indices after every step above), so
    # the point's tail -- its last failing frames finishing their 50 passes on
    # few tiles -- is paid once per point, as main.py pays it once per point
    whole = [v for v in args.point_snr.split(",") if v.strip()] if pgraph is None else []
    if whole and extra_slots is None:
        dec.close()
        extra_slots = max(64, (B // 4) // 64 * 64)
        dec = Decoder(graph, extra_slots)
        dec.mc_run(SEED, [1.0 / math.sqrt(2.0 * 10.0 ** (float(whole[0]) * 0.1))], 64, 1 << 40, args.iters,
                   static=False, split=args.split)
    base = (args.warmup + args.steps + len(extra)) * world * B
    for i, x in enumerate(whole):
        x = float(x)
        sg = 1.0 / math.sqrt(2.0 * 1.0 * (10.0 ** (x * 0.1)))
        PF = args.point_frames
        barrier(dist, local)
        t1 = time.perf_counter()
        c = dec.mc_run(SEED, [sg], PF, base + (i * world + rank) * PF, args.iters, static=False, split=args.split)
        c = allreduce_counters(dist, c, local)
        barrier(dist, local)
        dt = max_over_ranks(dist, time.perf_counter() - t1, local)
        f = int(c[0, 0])
        assert f == PF * world, (f, PF, world)
        snr_points.append({"snr_db": x, "scope": "point", "value": f / dt, "unit": "codewords/s",
                           "info_bits_per_s": f * k / dt, "ms": dt * 1e3, "frames": f, "schedule": "stream",
                           "slots": extra_slots, "avg_iters": int(c[0, 6]) / max(f, 1),
                           "fer": int(c[0, 1]) / max(f, 1), "ber": int(c[0, 2]) / (k * max(f, 1))})

    physical = None
    if args.phys_steps > 0 and pgraph is None and not ira_code:
        dec.close()
        physical = physical_extra(args, edd, graph, local, world, rank, dist, k)
    config4 = None
    if args.config4_snr.strip() and pgraph is None and not ira_code:
        dec.close()  # idempotent (the physical key may have closed it)
        config4 = config4_extra(args, local, world, rank, dist)
    config2 = config2_extra(args, local, world, rank, dist) if args.config2 and pgraph is None and not ira_code \
        else None
    config5 = config5_extra(args, local, world, rank, dist) if args.config5 and pgraph is None and not ira_code \
        else None
    dropin = dropin_extra(args, graph, n) if args.dropin_calls > 0 and pgraph is None else None

    frames_total = int(totals[0, 0])
    assert frames_total == B * world * args.steps, (frames_total, B, world, args.steps)
    iters_total = int(totals[0, 6])  # whole job
    cw_s = frames_total / elapsed

    # roofline of the dominant kernel (cn_kernel) on THIS rank: algorithmic
    # bytes = 16 B per edge per frame-iteration (read E_old + write E_new)
    cn_ms, cn_launches = prof["cn"]
    from ldpc_amd import _lib
    cn_name = _lib.lib().ldpc_cn_kernel_name(graph.handle).decode()
    vn_ms, vn_launches = prof["vn"]
    local_iters = int(local_totals[0, 6])  # this rank's frame-iterations
    cn_bytes_total = 16.0 * nnz * local_iters
    cn_avg_s = (cn_ms / 1e3) / max(cn_launches, 1)
    cn_bytes_per_launch = cn_bytes_total / max(cn_launches, 1)
    achieved = cn_bytes_per_launch / cn_avg_s / 1e9 if cn_launches else 0.0
    decode_ms = cn_ms + vn_ms
    # whole-decode algorithmic bytes: 8n + sum_iters 16 E + ceil(n/8) + 8 per frame
    frames_local = B * args.steps
    dec_bytes = frames_local * (8 * n + math.ceil(n / 8) + 8) + 16.0 * nnz * local_iters
    decode_gbs = dec_bytes / (decode_ms / 1e3) / 1e9 if decode_ms else 0.0
    traffic, traffic_src = committed_traffic(nnz, chunk)

    tile_ms, tile_launches = prof.get("tile", (0.0, 0))
    if tile_launches:  # tile-resident decoder: one launch decodes a chunk through all its iterations
        cn_name = _lib.lib().ldpc_tile_kernel_name(graph.handle).decode() or "tile_kernel"
        if args.schedule == "stream" and cn_name == "tile_kernel":
            cn_name = "tile_stream_kernel"  # the streaming Monte-Carlo variant of the same decoder
        # a streamed point's last frames finish on the split path's tail (cn + vn / vn_cols
        # launches): the whole decode's time is the tile launch's plus the tail's
        decode_ms = tile_ms + cn_ms + vn_ms + prof.get("vn_cols", (0.0, 0))[0]
        decode_gbs = dec_bytes / (decode_ms / 1e3) / 1e9 if decode_ms else 0.0
    out = {
        "metric": METRIC,
        "value": cw_s,
        "unit": "codewords/s",
        "info_bits_per_s": cw_s * k,
        "n_gpus": ranks_seen,
        "ranks_seen": ranks_seen,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (on-device Philox4x32-10 info bits, [u, A.u] codewords, BPSK/AWGN, reference "
                "channel model: noise std sigma^2, LLR 2y/sigma^2)",
        "config": {
            "workload": f"{args.code} SPA, max_iter {args.iters} + early termination, snr {args.snr} dB "
                        f"(reference axis, speed 1), {B} frames/GPU/step",
            "code": args.code, "n": n, "k": k, "edges_H_std": nnz, "max_iter": args.iters,
            "snr_db": args.snr, "frames_per_gpu": B, "global_batch": B * world,
            "parallelism": f"frame-sharded x{world}", "chunk_frames": chunk, "schedule": args.schedule,
        },
        "fer": totals[0, 1] / frames_total,
        "ber": totals[0, 2] / (k * frames_total),
        "avg_iters": iters_total / frames_total,
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
            "kernel": cn_name, "launches": cn_launches, "avg_launch_ms": cn_avg_s * 1e3,
            "bytes_per_launch": cn_bytes_per_launch,
            "bytes_model": "16 B x H_std edges x frame-iterations executed (E_old read + E_new write)",
        },
        "decode_roofline": {"achieved_GBs": decode_gbs, "frac": decode_gbs / HBM_PEAK_GBS,
                            "cn_ms": cn_ms, "vn_ms": vn_ms, "vn_cols_ms": prof.get("vn_cols", (0.0, 0))[0],
                            "tile_ms": tile_ms, "gen_ms": prof["generate"][0],
                            "count_ms": prof["count"][0]},
        "cpu_baseline": None,
    }
    if snr_points:
        out["snr_points"] = snr_points
    if physical is not None:
        out["physical"] = physical
    if config2 is not None:
        out["config2"] = config2
    if config4 is not None:
        out["config4"] = config4
    if config5 is not None:
        out["config5"] = config5
    if dropin is not None:
        out["dropin"] = dropin
    if not tile_launches and pgraph is None and cn_launches:
        # separate CN / VN launches: the roofline is the WHOLE decode, one "launch" = one
        # CN + one VN sweep over the resident slots; traffic = PMC bytes of the same pair
        out["cn_roofline"] = out["roofline"]
        tc, src_c = committed_traffic(nnz, chunk, "cn")
        tv, src_v = committed_traffic(nnz, chunk, "vn")
        read_bytes = frames_local * 8 * n + 8.0 * nnz * local_iters
        out["roofline"] = {
            "bound": "hbm", "achieved": decode_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": decode_gbs / HBM_PEAK_GBS,
            "traffic": (tc + tv) if (tc is not None and tv is not None) else None,
            "traffic_source": src_c if src_c == src_v else None,
            "kernel": f"{cn_name}+vn_kernel", "launches": cn_launches,
            "avg_launch_ms": decode_ms / cn_launches, "bytes_per_launch": dec_bytes / cn_launches,
            "bytes_model": "per frame 8 n (channel LLRs) + 16 B x H_std edges x iterations executed "
                           "(E_old read + E_new write) + ceil(n/8) + 8 (SURVEY 8d), over the CN + VN "
                           "launches' HIP-event time",
            "read_achieved": read_bytes / (decode_ms / 1e3) / 1e9,
            "read_frac": read_bytes / (decode_ms / 1e3) / 1e9 / HBM_PEAK_GBS,
        }
    if tile_launches and pgraph is None:
        # the whole decode is one kernel: algorithmic bytes per decoded frame
        # 8n + sum_iters 16 E + ceil(n/8) + 8, over this rank's frames, per launch
        out["roofline"] = {
            "bound": "hbm", "achieved": decode_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": decode_gbs / HBM_PEAK_GBS, "traffic": committed_traffic(nnz, chunk, "tile")[0],
            "traffic_source": committed_traffic(nnz, chunk, "tile")[1],
            "kernel": cn_name, "launches": tile_launches, "avg_launch_ms": tile_ms / tile_launches,
            "tail_ms": decode_ms - tile_ms, "bytes_per_launch": dec_bytes / tile_launches,
            "bytes_model": "per frame 8 n (channel LLRs) + 16 B x H_std edges x iterations executed "
                           "(E_old read + E_new write) + ceil(n/8) + 8 (SURVEY 8d); CN and VN fused",
        }
        # the north_star's "HBM-read roofline": the read part alone, 8 n + 8 B x edges x iterations
        read_bytes = frames_local * 8 * n + 8.0 * nnz * local_iters
        read_gbs = read_bytes / (decode_ms / 1e3) / 1e9 if decode_ms else 0.0
        out["roofline"]["read_achieved"] = read_gbs
        out["roofline"]["read_frac"] = read_gbs / HBM_PEAK_GBS
        # ... and in bytes the fabric actually read: the committed PMC read bytes per frame-iteration
        # (the same workload shape, tools/summarize_tile_profile.py) times this run's frame-iterations
        tsrc = out["roofline"]["traffic_source"]
        tj = json.load(open(os.path.join(ROOT, tsrc))) if tsrc else {}
        fil = tj.get("frame_iterations_per_launch")
        if fil and decode_ms:
            rd_fi = tj["kernels"]["tile"]["read_bytes"] / fil
            out["roofline"]["read_traffic_per_frame_iteration"] = rd_fi
            out["roofline"]["read_traffic_achieved"] = rd_fi * local_iters / (decode_ms / 1e3) / 1e9
            out["roofline"]["read_traffic_frac"] = out["roofline"]["read_traffic_achieved"] / HBM_PEAK_GBS
    if pgraph is not None:  # physical mode (not the reference's arithmetic: §8 f4)
        pnnz = int(pgraph.nnz)
        pms, pl = prof["phys"]
        cms, cl = prof["phys_cn"]
        vms, vl = prof["phys_vn"]
        where = "HBM-resident tiles" if cl else "LDS-resident"
        out["dtype"] = "f32"
        out["config"]["workload"] = out["config"]["workload"].replace(
            " SPA,", f" SPA physical mode (sparse H[:,perm], sign-consistent, fp32, {where}),")
        out["config"]["edges_H_phys"] = pnnz
        if ira_code:
            out["config"]["edges_H_std"] = None
            out["config"]["code_note"] = ("DVB-S2 rate-1/2 normal-frame profile (n=64800, degrees 8/3/2, check "
                                          "degree 7, staircase parity) with a seeded address table: ldpc_amd/ira.py")
        if cl:  # HBM tile path: phys_cn_tile dominates
            local_iters = int(local_totals[0, 6])
            cn_bytes = 12.0 * pnnz * local_iters
            cn_avg_s = (cms / 1e3) / cl
            achieved = cn_bytes / cl / cn_avg_s / 1e9
            out["roofline"] = {
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": None, "kernel": "phys_cn_tile_kernel",
                "launches": cl, "avg_launch_ms": cn_avg_s * 1e3, "bytes_per_launch": cn_bytes / cl,
                "bytes_model": "12 B x H edges x frame-iterations (L[col] gather + E_old read + E_new write, fp32)",
            }
            dec_bytes = (16.0 * pnnz + 12.0 * n) * local_iters
            out["decode_roofline"] = {"achieved_GBs": dec_bytes / ((cms + vms) / 1e3) / 1e9,
                                      "frac": dec_bytes / ((cms + vms) / 1e3) / 1e9 / HBM_PEAK_GBS,
                                      "phys_cn_ms": cms, "phys_vn_ms": vms, "gen_ms": prof["generate"][0],
                                      "count_ms": prof["count"][0]}
        else:
            from ldpc_amd import _lib
            pname = _lib.lib().ldpc_phys_kernel_name(pgraph.handle, 0).decode()
            out["roofline"] = {"bound": "valu", "kernel": pname, "launches": pl,
                               "avg_launch_ms": pms / max(pl, 1),
                               "note": "state in LDS; HBM traffic is the frame input only"}
            vi, vsrc = committed_valu(args.code, pname, args.snr)
            if vi and pms:
                # VALU issue roofline: wave-instructions per frame-iteration (committed PMC of the
                # same kernel and code) x this run's frame-iterations / the kernel's HIP-event time
                ach = vi * int(local_totals[0, 6]) / (pms / 1e3)
                out["roofline"].update({"achieved": ach, "peak": VALU_PEAK, "unit": "VALU wave-instr/s",
                                        "frac": ach / VALU_PEAK, "valu_insts_per_frame_iteration": vi,
                                        "valu_source": vsrc,
                                        "peak_model": "256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 "
                                                      "VALU instruction (MI355X_MICROARCH.md)"})
            out["decode_roofline"] = {"phys_ms": pms, "gen_ms": prof["generate"][0]}
        if rank == 0 and world == 1 and args.cpu_seconds > 0:
            out["cpu_baseline"] = cpu_baseline_phys((Hphys, H), k, args, ira_code)
    elif rank == 0 and world == 1 and args.cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline(H, k, args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.close()


if __name__ == "__main__":
    main()
