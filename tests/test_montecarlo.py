"""Monte-Carlo driver host logic (CPU): main.py semantics, sharding, one
all-reduce across ranks (gloo, world_size 2), results schema.

The per-rank counter source here is the CPU oracle (frames from the oracle's
restatement of the device frame source, decoded by the oracle) injected as
`counter_fn`, so the sharding / reduction code is exercised without a GPU;
the GPU path itself is covered by tests/test_gpu_mc.py.
"""
import json
import os
import socket

import numpy as np
import pytest

import oracle
from conftest import hstd_for
from ldpc_amd import montecarlo as mc
from ldpc_amd.results import SimulationResult

SEED = 20260213


def oracle_counter_fn(code, T, nllr=True):
    H = hstd_for(code)
    k = H.shape[1] - H.shape[0]

    def f(sigmas, count, frame0):
        out = []
        for p, s in enumerate(sigmas):
            u, _, llr = oracle.generate_frames(H, SEED, p, s, frame0, count)
            r = oracle.spa_decode(H, llr, T, nllr=nllr)
            out.append(oracle.main_counters(u, r["z"], r["status"], r["conv"],
                                            nllr_cnt=np.rint(r["nllr"] * k).astype(np.int64),
                                            iters=r["iters"]))
        return np.stack(out)
    return f


def test_snr_grid_matches_main_py():
    # main.py:193,206-209: ceil((end-start)/step)+1 points, clamped to end
    assert mc.snr_grid(0.0, 2.0, 1.0) == [0.0, 1.0, 2.0]
    assert mc.snr_grid(1.0, 4.0, 0.5) == [1.0, 1.5, 2.0, 2.5, 3.0, 3.5, 4.0]
    assert mc.snr_grid(0.0, 1.0, 0.3) == [0.0, 0.3, 0.6, 0.8999999999999999, 1.0]
    assert mc.snr_grid(2.0, 2.0, 1.0) == [2.0]


def test_sigma_matches_channel_py():
    import math
    for snr in (0.0, 1.0, 2.5):
        assert mc.sigma_for_snr(snr) == 1.0 / math.sqrt(2.0 * 1.0 * (10.0 ** (snr * 0.1)))


@pytest.mark.parametrize("total,world", [(10, 3), (65536, 8), (5, 8), (0, 2)])
def test_shard_partitions(total, world):
    seen = []
    for r in range(world):
        s, c = mc.shard(total, r, world)
        seen.extend(range(s, s + c))
    assert seen == list(range(total))


def test_point_results_follow_main_py():
    # 4 frames, k=10: failed 2 with 3+1 error bits; converged at 0 and 2
    c = np.array([[4, 2, 4, 2, 2, 6, 14, ]], dtype=np.int64)
    (p,) = mc.point_results(c, 10, [1.5], max_iter=7)
    assert p.fer == 0.5 and p.ber == 4 / 40 and p.avg_convergence_iterations == 1.0
    assert p.successful_blocks == 2 and p.failed_blocks == 2 and p.total_blocks == 4
    assert p.avg_normalized_llr == (6 / 10) / 4 and p.max_iterations == 7


def test_counters_equal_main_py_loop():
    """Oracle counters == a literal main.py-style per-frame loop (main.py:314-339)."""
    code, T = "BCH_7_4_1_strip", 10
    H = hstd_for(code)
    k = 4
    sig = mc.sigma_for_snr(1.0)
    u, _, llr = oracle.generate_frames(H, SEED, 0, sig, 0, 500)
    r = oracle.spa_decode(H, llr, T)
    failed = err = conv_sum = conv_cnt = 0
    for f in range(500):
        ok = r["status"][f] == 0
        failed += 0 if ok else 1
        if not ok:
            decoded = [int(b) ^ 1 for b in r["z"][f][:k]]
            err += sum(int(a) != b for a, b in zip(u[f], decoded))
        if r["conv"][f] >= 0:
            conv_sum += int(r["conv"][f])
            conv_cnt += 1
    got = oracle_counter_fn(code, T, nllr=False)([sig], 500, 0)[0]
    assert list(got[:5]) == [500, failed, err, conv_sum, conv_cnt]


def test_single_rank_sweep_uses_counter_fn():
    f = oracle_counter_fn("BCH_7_4_1_strip", 5)
    ctr = mc.run_sweep(None, [0.0, 2.0], 300, 5, counter_fn=f)
    assert ctr.shape == (2, 7) and (ctr[:, 0] == 300).all()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def gloo_allreduce(arr):
    """ONE all-reduce of the counter matrix over the default (gloo) process
    group: the CPU stand-in for ldpc_amd.comm.Comm.allreduce (RCCL)."""
    import torch
    import torch.distributed as dist
    t = torch.from_numpy(np.ascontiguousarray(arr).reshape(-1).copy())
    dist.all_reduce(t)
    return t.numpy().reshape(arr.shape)


def _rank_main(rank, world, port, outdir):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        f = oracle_counter_fn("wimax_576_0.5", 4)
        ctr = mc.run_sweep(None, [0.0, 1.5, 3.0], 37, 4, rank=rank, world=world,
                           allreduce=gloo_allreduce, counter_fn=f)
        np.save(os.path.join(outdir, f"rank{rank}.npy"), ctr)
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_sweep_equals_single_rank(tmp_path):
    """world_size 2 over gloo: disjoint frame shards + ONE all-reduce == 1 rank."""
    import torch.multiprocessing as tmp
    port = _free_port()
    tmp.spawn(_rank_main, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    a = np.load(tmp_path / "rank0.npy")
    b = np.load(tmp_path / "rank1.npy")
    np.testing.assert_array_equal(a, b)  # every rank holds the reduced counters
    single = mc.run_sweep(None, [0.0, 1.5, 3.0], 37, 4, counter_fn=oracle_counter_fn("wimax_576_0.5", 4))
    np.testing.assert_array_equal(a, single)
    assert (a[:, 0] == 37).all()


def test_results_json_csv_roundtrip(tmp_path):
    pts = mc.point_results(np.array([[10, 3, 5, 4, 7, 0, 30], [10, 0, 0, 0, 10, 0, 10]]), 288, [0.0, 1.0],
                           matrix_path="wimax_576_0.5", max_iter=5)
    from ldpc_amd.results import SimulationConfig
    cfg = SimulationConfig(matrix_path="m", n=576, m=288, k=288, rate=0.5, blocks=10, max_iterations=5,
                           encoding_method="standard", interleaver_type="none", decoder_type="sumproduct",
                           channel_mode=1, modulation=1, speed=1.0, snr_range=(0.0, 1.0, 1.0), threads=1,
                           timestamp="t")
    res = SimulationResult(config=cfg, snr_points=pts, wall_clock_seconds=1.5)
    res.to_json(tmp_path / "r.json")
    back = SimulationResult.from_json(tmp_path / "r.json")
    assert back == res
    res.to_csv(tmp_path / "r.csv")
    lines = open(tmp_path / "r.csv").read().splitlines()
    assert lines[0].split(",")[:4] == ["snr_db", "ber", "fer", "avg_normalized_llr"] and len(lines) == 3


def test_reads_reference_results_file():
    """Our loader reads the reference's committed results.json (schema parity)."""
    path = "/root/reference/python_ldpc_app/results.json"
    if not os.path.exists(path):
        pytest.skip("reference tree not present (GPU box)")
    r = SimulationResult.from_json(path)
    raw = json.load(open(path))
    assert len(r.snr_points) == len(raw["snr_points"])
    assert r.snr_points[0].fer == raw["snr_points"][0]["fer"]
