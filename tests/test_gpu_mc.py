"""On-device frame source and Monte-Carlo counters.

- generator vs its CPU restatement (oracle/channel_oracle.c): info bits
  bit-exact, LLRs to the ulp of log/cos/sin;
- generated codewords satisfy H_std c = 0 (checked through the bits);
- ldpc_mc_run counters == main.py counter semantics applied to the oracle's
  decode of the very same device-generated frames;
- frame-index sharding: counters of [0,B) == counters of [0,B/2) + [B/2,B)
  (what the multi-GPU run relies on).
"""
import numpy as np
import pytest

import oracle
from conftest import hstd_for

pytestmark = pytest.mark.gpu

SEED = 20260213


def _decoder(code, frames):
    from ldpc_amd.device import Decoder, Graph
    return Decoder(Graph.cached(hstd_for(code)), frames)


@pytest.mark.parametrize("code", ["BCH_7_4_1_strip", "wimax_576_0.5", "wimax_2304_0.5", "wimax_2304_0.75A"])
def test_generator_matches_cpu_restatement(gpu_available, code):
    H = hstd_for(code)
    dec = _decoder(code, 96)
    sigma = oracle.sigma_for_snr(2.0)
    u, llr = dec.generate(SEED, 3, sigma, 1000, 96)
    uo, co, lo = oracle.generate_frames(H, SEED, 3, sigma, 1000, 96)
    np.testing.assert_array_equal(u, uo)
    np.testing.assert_allclose(llr, lo, rtol=1e-12, atol=1e-12)
    # the codeword the CPU restatement encoded satisfies H_std c = 0
    assert not ((H @ co.T.astype(np.int64)) % 2).any()


def test_generator_statistics(gpu_available):
    """LLR = 2(x + s^2 g)/s^2: mean +-2/s^2, std 2 (channel.py:68-80)."""
    code = "wimax_576_0.5"
    dec = _decoder(code, 512)
    sigma = oracle.sigma_for_snr(1.0)
    u, llr = dec.generate(SEED, 0, sigma, 0, 512)
    _, c, _ = oracle.generate_frames(hstd_for(code), SEED, 0, sigma, 0, 512)
    x = 2.0 * c - 1.0
    s2 = sigma ** 2
    noise = (llr * s2 / 2.0 - x) / s2
    assert abs(noise.mean()) < 0.01
    assert abs(noise.std() - 1.0) < 0.01
    assert abs(u.mean() - 0.5) < 0.01


@pytest.mark.parametrize("code,T,snrs,B", [
    ("wimax_576_0.5", 10, [0.0, 1.5, 3.0], 192),
    ("BCH_7_4_1_strip", 10, [0.0, 4.0], 4096),
])
def test_mc_counters_match_oracle(gpu_available, code, T, snrs, B):
    H = hstd_for(code)
    dec = _decoder(code, B)
    sig = [oracle.sigma_for_snr(s) for s in snrs]
    ctr = dec.mc_run(SEED, sig, B, 0, T, nllr=True)
    k = H.shape[1] - H.shape[0]
    for p, s in enumerate(sig):
        u, llr = dec.generate(SEED, p, s, 0, B)
        o = oracle.spa_decode(H, llr, T, nllr=True)
        want = oracle.main_counters(u, o["z"], o["status"], o["conv"],
                                    nllr_cnt=np.rint(o["nllr"] * k).astype(np.int64), iters=o["iters"])
        np.testing.assert_array_equal(ctr[p], want)


def test_mc_sharding_is_additive(gpu_available):
    code = "wimax_576_0.5"
    dec = _decoder(code, 256)
    sig = [oracle.sigma_for_snr(2.0)]
    whole = dec.mc_run(SEED, sig, 256, 0, 8)
    a = dec.mc_run(SEED, sig, 128, 0, 8)
    b = dec.mc_run(SEED, sig, 128, 128, 8)
    np.testing.assert_array_equal(whole, a + b)


def test_simulate_end_to_end_results_schema(gpu_available, tmp_path):
    """montecarlo.simulate: GPU sweep -> reference results schema, counters == oracle."""
    from ldpc_amd import montecarlo as mc
    from ldpc_amd.results import SimulationResult
    snrs = mc.snr_grid(0.0, 2.0, 1.0)
    res, ctr = mc.simulate("BCH_7_4_1_strip", snrs, 2000, 10)
    H = hstd_for("BCH_7_4_1_strip")
    for p, s in enumerate(snrs):
        u, _, llr = oracle.generate_frames(H, SEED, p, mc.sigma_for_snr(s), 0, 2000)
        o = oracle.spa_decode(H, llr, 10)
        want = oracle.main_counters(u, o["z"], o["status"], o["conv"], iters=o["iters"])
        np.testing.assert_array_equal(ctr[p][[0, 1, 2, 3, 4, 6]], want[[0, 1, 2, 3, 4, 6]])
    res.to_json(tmp_path / "r.json")
    back = SimulationResult.from_json(tmp_path / "r.json")
    assert [sp.fer for sp in back.snr_points] == [sp.fer for sp in res.snr_points]


# --- streaming schedule (slots refilled as frames stop) vs the static chunks
@pytest.mark.parametrize("code,cap,frames,T,snrs", [
    ("wimax_576_0.5", 256, 2048, 20, [1.0, 2.0, 3.0]),       # ~8 frames per slot, mixed iteration counts
    ("BCH_7_4_1_strip", 64, 5000, 10, [0.0, 3.0, 6.0]),       # ragged last refill, frames >> slots
    ("wimax_2304_0.75A", 128, 384, 12, [2.0, 4.0]),           # odd-degree sign quirk: failures at 4 dB
    ("wimax_576_0.5", 512, 100, 50, [0.0]),                   # fewer frames than slots (one partial tile)
])
def test_stream_counters_equal_static(gpu_available, code, cap, frames, T, snrs):
    dec = _decoder(code, cap)
    sig = [oracle.sigma_for_snr(s) for s in snrs]
    stream = dec.mc_run(SEED, sig, frames, 7, T, nllr=True)
    static = dec.mc_run(SEED, sig, frames, 7, T, nllr=True, static=True)
    np.testing.assert_array_equal(stream, static)
    assert (stream[:, 0] == frames).all()


def test_stream_refills_match_oracle(gpu_available):
    """Slots decode several frames each; counters == oracle on the same frames."""
    code, cap, frames, T = "wimax_576_0.5", 128, 640, 10
    H = hstd_for(code)
    k = H.shape[1] - H.shape[0]
    sig = [oracle.sigma_for_snr(2.0)]
    ctr = _decoder(code, cap).mc_run(SEED, sig, frames, 0, T, nllr=True)
    u, llr = _decoder(code, frames).generate(SEED, 0, sig[0], 0, frames)
    o = oracle.spa_decode(H, llr, T, nllr=True)
    want = oracle.main_counters(u, o["z"], o["status"], o["conv"],
                                nllr_cnt=np.rint(o["nllr"] * k).astype(np.int64), iters=o["iters"])
    np.testing.assert_array_equal(ctr[0], want)


def test_stream_zero_frames(gpu_available):
    dec = _decoder("BCH_7_4_1_strip", 64)
    ctr = dec.mc_run(SEED, [oracle.sigma_for_snr(1.0)], 0, 0, 10)
    assert not ctr.any()


# The streaming schedule on tile-capable graphs runs inside the tile-resident
# decoder (tile_stream_kernel: per-lane refill between passes); LDPC_F_SPLIT
# keeps the per-iteration CN/VN/refill loop.  Same frames, same counters.
@pytest.mark.parametrize("code,cap,frames,T,snrs", [
    ("wimax_576_0.5", 192, 1000, 12, (0.0, 2.0, 3.5)),
    ("wimax_576_0.5", 64, 333, 50, (2.5,)),
    ("BCH_7_4_1_strip", 64, 5000, 10, (0.0, 4.0)),
    ("wimax_576_0.5", 128, 130, 1, (1.0, 6.0)),     # max_iter 1: every frame stops after its first pass
    ("wimax_576_0.5", 4096, 70, 8, (0.5,)),         # far fewer frames than slots (idle workgroups)
    ("wimax_2304_0.5", 256, 700, 12, (1.0, 3.0)),   # 16-frame sub-tiles (tile_sub_stream_kernel)
    ("wimax_2304_0.5", 64, 150, 1, (2.0,)),         # sub-tiles, max_iter 1
    ("wimax_2304_0.75A", 256, 700, 12, (2.0, 3.5)),  # 8-frame sub-tiles (tile8_stream_kernel, K = 8)
    ("wimax_2304_0.75B", 64, 150, 1, (2.0,)),        # tile8 streaming, max_iter 1
    ("wimax_2304_0.75A", 4096, 70, 8, (3.0,)),       # far fewer frames than slots
])
def test_tile_stream_equals_split_stream(gpu_available, code, cap, frames, T, snrs, monkeypatch):
    monkeypatch.setenv("LDPC_HANDOFF", "0")  # the whole point in the tile kernel (hand-off: next test)
    dec = _decoder(code, cap)
    sig = [oracle.sigma_for_snr(s) for s in snrs]
    dec.profile(True)
    a = dec.mc_run(SEED, sig, frames, 3, T, nllr=True)
    p = dec.profile_read()
    dec.profile(False)
    assert p["tile"][1] == len(snrs) and p["cn"][1] == 0, p  # one tile launch per point
    b = dec.mc_run(SEED, sig, frames, 3, T, nllr=True, split=True)
    np.testing.assert_array_equal(a, b)
    assert (a[:, 0] == frames).all()


@pytest.mark.parametrize("at", [None, "8"])
def test_stream_tail_compaction_keeps_counters(gpu_available, monkeypatch, at):
    """The split streaming schedule compacts its tail (frames still running once
    the supply is out move into the first tiles): counters equal the
    uncompacted stream and the static schedule -- also compacting whenever a
    tile can be dropped (LDPC_COMPACT_AT=8)."""
    code, cap, frames, T = "wimax_2304_0.5", 256, 1500, 20
    dec = _decoder(code, cap)
    sig = [oracle.sigma_for_snr(s) for s in (2.5, 3.0)]
    if at:
        monkeypatch.setenv("LDPC_COMPACT_AT", at)
    a = dec.mc_run(SEED, sig, frames, 11, T, nllr=True, split=True)
    monkeypatch.setenv("LDPC_COMPACT", "0")
    b = dec.mc_run(SEED, sig, frames, 11, T, nllr=True, split=True)
    monkeypatch.delenv("LDPC_COMPACT")
    c = dec.mc_run(SEED, sig, frames, 11, T, nllr=True, static=True)
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(a, c)
    assert (a[:, 0] == frames).all()


def test_fit_slots_caps_the_workspace(gpu_available):
    """A batch whose fp64 state exceeds the HBM budget streams through fewer
    slots (wimax_2304_0.5: 5.3 MB per frame)."""
    from ldpc_amd.device import Decoder, Graph
    g = Graph.cached(hstd_for("wimax_2304_0.5"))
    assert Decoder.fit_slots(g, 65536) < 65536  # 348 GB of messages > the 160 GB default
    slots = Decoder.fit_slots(g, 65536, budget=3e9)
    assert slots % 64 == 0 and 64 <= slots < 1024
    assert Decoder.workspace_bytes(g, slots) <= 3e9
    assert Decoder.fit_slots(Graph.cached(hstd_for("wimax_576_0.5")), 65536) == 65536
    dec = Decoder(g, slots)
    ctr = dec.mc_run(SEED, [oracle.sigma_for_snr(3.0)], 3 * slots + 5, 0, 6)
    assert ctr[0, 0] == 3 * slots + 5


@pytest.mark.parametrize("code,handoff", [("wimax_2304_0.5", "256"), ("wimax_2304_0.5", "20"),
                                          ("wimax_2304_0.75A", "256"), ("wimax_2304_0.75A", "20")])
def test_stream_handoff_keeps_counters(gpu_available, monkeypatch, code, handoff):
    """The streaming sub-tile kernels (16-frame tile_sub_stream_kernel, 8-frame
    tile8_stream_kernel) hand their last running frames to the split path's
    column-parallel tail (launch_vn_tail) once the supply is out: the counters
    equal the sub-tile kernel draining alone, the static schedule and the
    split stream with the per-tile vn_kernel."""
    cap, frames, T = 256, 1500, 20
    dec = _decoder(code, cap)
    sig = [oracle.sigma_for_snr(s) for s in (2.5, 3.0)]
    monkeypatch.setenv("LDPC_HANDOFF", handoff)
    dec.profile(True)
    a = dec.mc_run(SEED, sig, frames, 11, T, nllr=True)
    p = dec.profile_read()
    dec.profile(False)
    assert p["tile"][1] == 2, p
    # with 256 (every slot) the kernel hands off as soon as the supply is out,
    # so the tail always runs; with 20 it runs only if some workgroup still
    # holds a running frame when at most 20 are left -- timing-dependent (the
    # last frames may all stop in the same pass), so only the counters are held
    if handoff == "256":
        assert p["cn"][1] > 0, p  # the tail ran on the split path
    monkeypatch.setenv("LDPC_HANDOFF", "0")
    b = dec.mc_run(SEED, sig, frames, 11, T, nllr=True)
    c = dec.mc_run(SEED, sig, frames, 11, T, nllr=True, static=True)
    monkeypatch.setenv("LDPC_TAIL_VN", "0")
    d = dec.mc_run(SEED, sig, frames, 11, T, nllr=True, split=True)
    monkeypatch.delenv("LDPC_TAIL_VN")
    e = dec.mc_run(SEED, sig, frames, 11, T, nllr=True, split=True)
    for x in (b, c, d, e):
        np.testing.assert_array_equal(a, x)
    assert (a[:, 0] == frames).all()


def test_tile8_stream_matches_oracle_config4(gpu_available):
    """Config 4's decoder: the 8-frame streaming kernel on wimax_2304_0.75A at
    T=50 (the bench's config4 sweep runs exactly this call), frames through 64
    slots so that every slot decodes several; counters == the oracle's
    main.py counters on the very frames the device generated, per point."""
    code, cap, frames, T = "wimax_2304_0.75A", 64, 96, 50
    H = hstd_for(code)
    k = H.shape[1] - H.shape[0]
    snrs = (2.5, 3.0, 4.0)
    sig = [oracle.sigma_for_snr(s) for s in snrs]
    dec = _decoder(code, cap)
    dec.profile(True)
    ctr = dec.mc_run(SEED, sig, frames, 5000, T, nllr=True)
    p = dec.profile_read()
    dec.profile(False)
    assert p["tile"][1] == len(snrs), p  # one tile8_stream_kernel launch per point
    # ... which handed its last running frames to the split path's tail
    # (cn_sub_kernel stream form + vn_cols_kernel + tail_exit_kernel)
    assert p["cn"][1] > 0 and p["vn_cols"][1] > 0, p
    gen = _decoder(code, frames)
    for i, sg in enumerate(sig):
        u, llr = gen.generate(SEED, i, sg, 5000, frames)
        o = oracle.spa_decode(H, llr, T, nllr=True)
        want = oracle.main_counters(u, o["z"], o["status"], o["conv"],
                                    nllr_cnt=np.rint(o["nllr"] * k).astype(np.int64), iters=o["iters"])
        np.testing.assert_array_equal(ctr[i], want, err_msg=f"{snrs[i]} dB")


@pytest.mark.parametrize("snr", [2.5, 3.0])
def test_sub_stream_handoff_matches_oracle(gpu_available, snr):
    """The headline code's streaming path end to end against the oracle:
    tile_sub_stream_kernel (16-frame sub-tiles) -> hand-off at supply end ->
    the split tail (cn_sub_kernel's stream form + vn_cols_kernel +
    tail_exit_kernel), 192 frames through 64 slots at T = 50, so the tail
    carries frames that started in the stream kernel; counters == the
    oracle's main.py counters on the very frames the device generated."""
    code, cap, frames, T = "wimax_2304_0.5", 64, 192, 50
    H = hstd_for(code)
    k = H.shape[1] - H.shape[0]
    sg = oracle.sigma_for_snr(snr)
    dec = _decoder(code, cap)
    dec.profile(True)
    ctr = dec.mc_run(SEED, [sg], frames, 7000, T, nllr=True)
    p = dec.profile_read()
    dec.profile(False)
    assert p["tile"][1] == 1, p  # one tile_sub_stream_kernel launch
    assert p["cn"][1] > 0 and p["vn_cols"][1] > 0, p  # the split tail ran
    u, llr = _decoder(code, frames).generate(SEED, 0, sg, 7000, frames)
    o = oracle.spa_decode(H, llr, T, nllr=True)
    want = oracle.main_counters(u, o["z"], o["status"], o["conv"],
                                nllr_cnt=np.rint(o["nllr"] * k).astype(np.int64), iters=o["iters"])
    np.testing.assert_array_equal(ctr[0], want)


def test_tile8_stream_r12_equals_static(gpu_available, monkeypatch):
    """tile8's L_A-in-LDS variant (wimax_2304_0.5 with LDPC_TILE8=1): the
    streaming kernel (L_A reloaded from ch for refilled slots) == its static
    schedule == the default graph's tile_sub decoders."""
    from ldpc_amd.device import Decoder, Graph
    code, cap, frames, T = "wimax_2304_0.5", 128, 400, 15
    sig = [oracle.sigma_for_snr(s) for s in (1.5, 3.0)]
    monkeypatch.setenv("LDPC_TILE8", "1")
    g8 = Graph(hstd_for(code))
    monkeypatch.delenv("LDPC_TILE8")
    d8 = Decoder(g8, cap)
    monkeypatch.setenv("LDPC_HANDOFF", "0")
    a = d8.mc_run(SEED, sig, frames, 9, T, nllr=True)
    monkeypatch.delenv("LDPC_HANDOFF")
    b = d8.mc_run(SEED, sig, frames, 9, T, nllr=True)  # with the hand-off to the split tail
    c = d8.mc_run(SEED, sig, frames, 9, T, nllr=True, static=True)
    d = _decoder(code, cap).mc_run(SEED, sig, frames, 9, T, nllr=True)
    for x in (b, c, d):
        np.testing.assert_array_equal(a, x)


@pytest.mark.parametrize("code,cap,frames,T,snrs", [
    ("wimax_2304_0.5", 256, 1500, 20, (2.5, 3.0)),    # tile_sub_stream_kernel + hand-off
    ("wimax_2304_0.75A", 128, 700, 20, (3.0, 4.0)),   # tile8_stream_kernel + hand-off
    ("wimax_576_0.5", 128, 2000, 30, (1.5, 2.5)),     # tile_stream_kernel
])
def test_supply_order_keeps_counters(gpu_available, monkeypatch, code, cap, frames, T, snrs):
    """Longest job first (frame_order.hip: frames enter the slots in descending
    syndrome weight of their hard decisions) changes only WHEN a frame is
    decoded: the counters equal frame-index order (LDPC_LPT=0), the split
    streaming loop under the same order, and the static schedule."""
    dec = _decoder(code, cap)
    sig = [oracle.sigma_for_snr(s) for s in snrs]
    a = dec.mc_run(SEED, sig, frames, 21, T, nllr=True)
    b = dec.mc_run(SEED, sig, frames, 21, T, nllr=True, split=True)
    monkeypatch.setenv("LDPC_LPT", "0")
    c = dec.mc_run(SEED, sig, frames, 21, T, nllr=True)
    monkeypatch.delenv("LDPC_LPT")
    d = dec.mc_run(SEED, sig, frames, 21, T, nllr=True, static=True)
    for x in (b, c, d):
        np.testing.assert_array_equal(a, x)
    assert (a[:, 0] == frames).all()


@pytest.mark.parametrize("code,snr,count", [("wimax_2304_0.5", 3.0, 700), ("wimax_2304_0.75A", 2.5, 300),
                                            ("wimax_576_0.5", 1.0, 1000)])
def test_frame_order_matches_host_ranking(gpu_available, code, snr, count):
    """frame_order.hip's supply order == the stable descending ranking by the
    syndrome weight of H_std (llr > 0) and, for equal weights on graphs with
    at most half the rows of odd degree, the least reliable identity bit of an
    odd-degree row first -- recomputed on the host from the oracle's
    restatement of the device frame source (oracle/channel_oracle.c)."""
    H = hstd_for(code).tocsr()
    m, n = H.shape
    sig = oracle.sigma_for_snr(snr)
    frame0 = 123457
    order = _decoder(code, 64).frame_order(SEED, 2, sig, frame0, count)
    _, _, llr = oracle.generate_frames(H, SEED, 2, sig, frame0, count)
    hard = (llr > 0.0).astype(np.int64)
    w = np.asarray(((H @ hard.T) % 2).sum(axis=0)).ravel().astype(np.uint64)
    odd = (np.diff(H.indptr) % 2) == 1
    key = w << np.uint64(16)
    if 2 * odd.sum() <= m:
        weak = np.abs(llr[:, n - m:][:, odd]).astype(np.float32).min(axis=1)
        key |= np.uint64(0xFFFF) - (weak.view(np.uint32) >> 15).astype(np.uint64)
    want = np.argsort(-key.astype(np.int64), kind="stable")
    np.testing.assert_array_equal(order, want)
    assert w[order[0]] >= w[order[-1]]
