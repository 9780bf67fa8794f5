"""BER/FER Monte-Carlo sweep on the GPU(s) -- the caller of the hot path.

Reproduces the counter semantics of python_ldpc_app/main.py:run_simulation
(:178-442) with the frame pipeline on the device (ldpc_mc_run):
  * SNR grid: steps = ceil((end-start)/step) + 1, each point clamped to `end`
    (main.py:193, :206-209); sigma = 1/sqrt(2*speed*10^(snr/10)) (channel.py:113);
  * per frame: Result OK <=> syndrome zero; error bits counted only in frames
    whose decode FAILED (main.py:130-138); convergence iteration summed over
    converged frames (:154-172);
  * per point: FER = failed/B, BER = err/(k*B), avg_conv = sum/count,
    avg normalized LLR = sum/B (:346-369).
Multi-GPU (one process per GPU): rank r decodes the global frame indices
[r*B/W, (r+1)*B/W) of every SNR point -- the Philox stream is keyed by the
global index, so the counters are identical for any W -- and the whole
[points x 7] counter matrix is summed with ONE all-reduce: RCCL over xGMI
through the C ABI (ldpc_amd.comm, no PyTorch); the CPU tests inject a gloo
reducer of their own (tests/test_montecarlo.py) to exercise the same sharding
logic.
"""
import argparse
import math
import os
import time
from datetime import datetime

import numpy as np

from .results import SimulationConfig, SimulationResult, SNRPointResult

NCOUNT = 7  # frames, failed, err_bits, sum_conv, n_conv, sum_nllr_count, iters


def snr_grid(initial, end, step):
    """main.py:193,206-209."""
    steps = int(math.ceil((end - initial) / step)) + 1
    out = []
    for s in range(steps):
        v = initial + s * step
        out.append(end if v > end else v)
    return out


def sigma_for_snr(snr_db, speed=1.0):
    """channel.py:113 (mode 1)."""
    return 1.0 / math.sqrt(2.0 * speed * (10.0 ** (snr_db * 0.1)))


def shard(total, rank, world):
    """Balanced contiguous split of [0, total) -> (start, count) for `rank`."""
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def point_results(counters, k, snrs, matrix_path="", max_iter=5):
    """Per-SNR SNRPointResult from the summed counter matrix (main.py:346-389)."""
    pts = []
    for snr, c in zip(snrs, counters):
        frames, failed, err, sconv, nconv, snllr = (int(x) for x in c[:6])
        pts.append(SNRPointResult(
            snr_db=float(snr),
            ber=(err / (k * frames)) if k * frames > 0 else 0.0,
            fer=failed / frames if frames else 0.0,
            avg_normalized_llr=(snllr / k) / frames if frames and k else 0.0,
            total_blocks=frames, successful_blocks=frames - failed, failed_blocks=failed,
            avg_convergence_iterations=(sconv / nconv) if nconv else 0.0,
            matrix_path=matrix_path, max_iterations=max_iter))
    return pts


def run_sweep(decoder, snrs, blocks, max_iter, seed=20260213, nllr=False, speed=1.0,
              rank=0, world=1, allreduce=None, counter_fn=None):
    """Counters [len(snrs), 7] for `blocks` frames per SNR point, summed over ranks.

    decoder     ldpc_amd.device.Decoder (its graph fixes the code) -- or None with counter_fn
    counter_fn  (sigmas, count, frame0) -> int64 [points, 7]; defaults to
                decoder.mc_run (the GPU path).  Tests inject a CPU stand-in to
                exercise the sharding/all-reduce logic without a GPU.
    allreduce   callable(np.ndarray int64) -> summed array (ldpc_amd.comm.Comm.allreduce)
    """
    sig = [sigma_for_snr(s, speed) for s in snrs]
    start, count = shard(int(blocks), rank, world)
    if counter_fn is None:
        def counter_fn(sigmas, cnt, frame0):
            return decoder.mc_run(seed, sigmas, cnt, frame0, max_iter, nllr=nllr)
    local = np.asarray(counter_fn(sig, count, start), dtype=np.int64).reshape(len(snrs), NCOUNT)
    if world > 1:
        if allreduce is None:
            raise ValueError("world > 1 needs an allreduce")
        local = np.asarray(allreduce(local), dtype=np.int64).reshape(len(snrs), NCOUNT)
    return local


def simulate(matrix, snrs, blocks, max_iter, seed=20260213, nllr=False, chunk=65536, device=0,
             rank=0, world=1, allreduce=None, matrix_path=""):
    """Full sweep on this process's GPU -> SimulationResult (reference schema)."""
    from .code import EncoderDecoderData, load_committed_code
    from .device import Decoder, Graph
    t0 = time.time()
    if isinstance(matrix, EncoderDecoderData):
        edd = matrix
    elif isinstance(matrix, str) and os.path.exists(matrix):
        edd = EncoderDecoderData(matrix)
    else:
        edd = load_committed_code(matrix)
    g = Graph(edd._h_std, device=device)
    dec = Decoder(g, Decoder.fit_slots(g, min(max(1, shard(int(blocks), rank, world)[1]), chunk)))
    ctr = run_sweep(dec, snrs, blocks, max_iter, seed=seed, nllr=nllr, rank=rank, world=world,
                    allreduce=allreduce)
    pts = point_results(ctr, edd._k, snrs, matrix_path=matrix_path or str(matrix), max_iter=max_iter)
    cfg = SimulationConfig(
        matrix_path=matrix_path or str(matrix), n=edd._n, m=edd._m, k=edd._k, rate=edd._rate,
        blocks=int(blocks), max_iterations=int(max_iter), encoding_method="standard",
        interleaver_type="none", decoder_type="sumproduct", channel_mode=1, modulation=1,
        speed=1.0, snr_range=(snrs[0], snrs[-1], (snrs[1] - snrs[0]) if len(snrs) > 1 else 0.0),
        threads=world, timestamp=datetime.now().isoformat())
    return SimulationResult(config=cfg, snr_points=pts, wall_clock_seconds=time.time() - t0), ctr


def main(argv=None):
    ap = argparse.ArgumentParser(description="GPU BER/FER sweep (main.py semantics, AWGN mode 1, BPSK)")
    ap.add_argument("--matrix", required=True, help="ALIST path or a committed code name")
    ap.add_argument("-b", "--blocks", type=int, default=1000)
    ap.add_argument("-i", "--iterations", type=int, default=5)
    ap.add_argument("--initial-snr", type=float, default=0.0)
    ap.add_argument("--end-snr", type=float, default=3.0)
    ap.add_argument("--step-snr", type=float, default=1.0)
    ap.add_argument("--normalized-llr", action="store_true")
    ap.add_argument("--seed", type=int, default=20260213)
    ap.add_argument("--output-json")
    ap.add_argument("--output-csv")
    a = ap.parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    allreduce = comm = None
    if world > 1:
        from .comm import Comm
        comm = Comm.from_env(local)
        allreduce = comm.allreduce
    snrs = snr_grid(a.initial_snr, a.end_snr, a.step_snr)
    res, _ = simulate(a.matrix, snrs, a.blocks, a.iterations, seed=a.seed, nllr=a.normalized_llr,
                      device=local, rank=rank, world=world, allreduce=allreduce)
    if rank == 0:
        for sp in res.snr_points:
            print(f"SNR {sp.snr_db:.2f} dB  FER {sp.fer:.6f}  BER {sp.ber:.6e}  "
                  f"ok {sp.successful_blocks}/{sp.total_blocks}  avg conv {sp.avg_convergence_iterations:.3f}")
        if a.output_json:
            res.to_json(a.output_json)
        if a.output_csv:
            res.to_csv(a.output_csv)
    if comm is not None:
        comm.close()


if __name__ == "__main__":
    main()
