"""The exact timed path of the headline (BASELINE config 3) against the oracle.

bench.py's step is `Decoder.mc_run(SEED, [sigma], B, frame0, 50, static=True)`
on wimax_2304_0.5: on-device generate -> tile_sub_kernel<4> (all 50
iterations with early termination in one launch) -> count_kernel.  Here the
same call, at a frame offset inside a later 32,768-frame step, is compared
counter for counter with the oracle's decode of the very frames the device
generated (main.py:130-138,154-172 semantics, oracle.main_counters), and the
per-frame hard decisions / convergence iteration / Result of the drop-in
decode of those LLRs with the oracle's.  1 dB is the timed point (every frame
runs 50 saturating iterations: where an ulp of atanh could flip a decision);
2 and 3 dB are bench's extra points.
"""
import numpy as np
import pytest

import oracle
from conftest import assert_llr_close, hstd_for

pytestmark = pytest.mark.gpu

SEED = 20260213  # bench.py SEED
CODE = "wimax_2304_0.5"
T = 50
STEP = 32768  # bench.py --frames


def _decoder(frames):
    from ldpc_amd.device import Decoder, Graph
    return Decoder(Graph.cached(hstd_for(CODE)), frames)


def _want(H, u, llr):
    o = oracle.spa_decode(H, llr, T)
    return o, oracle.main_counters(u, o["z"], o["status"], o["conv"], iters=o["iters"])


@pytest.mark.parametrize("snr,step", [(1.0, 3), (1.0, 7), (2.0, 5), (3.0, 6)])
def test_bench_step_counters_equal_oracle(gpu_available, snr, step, monkeypatch):
    """One bench step's call (one SNR point per call, snr_point 0), 64 frames.
    The bench's 512-tile chunks run the sub-tile decoder; so does this 1-tile
    call once the small-batch column-parallel path is off (LDPC_SMALL_COLS=0)."""
    monkeypatch.setenv("LDPC_SMALL_COLS", "0")
    H = hstd_for(CODE)
    B = 64
    frame0 = STEP * step + 1000 * step
    dec = _decoder(B)
    sig = oracle.sigma_for_snr(snr)
    dec.profile(True)
    ctr = dec.mc_run(SEED, [sig], B, frame0, T, static=True)
    prof = dec.profile_read()
    dec.profile(False)
    assert prof["tile"][1] == 1 and prof["cn"][1] == 0, prof  # the fused sub-tile decoder ran, once
    u, llr = dec.generate(SEED, 0, sig, frame0, B)
    o, want = _want(H, u, llr)
    np.testing.assert_array_equal(ctr[0], want)
    r = dec.decode(llr, T, post=True)
    np.testing.assert_array_equal(r.z, o["z"])
    np.testing.assert_array_equal(r.conv, o["conv"])
    np.testing.assert_array_equal(r.status, o["status"])
    # frames that run all T iterations without converging (FER 3.5 % at 3 dB)
    # can amplify one ulp of a message tens of thousands of times; where the
    # oracle itself moves that far under one ulp of tanh, that is the bound
    # (oracle.conditioning_slack, as tests/test_gpu_parity.py)
    sl_L, _ = oracle.conditioning_slack(H, llr, T)
    assert_llr_close(r.post, o["post"], f"posterior L at {snr} dB", slack=sl_L)


def test_three_point_call_equals_oracle(gpu_available):
    """The VERDICT r2 form: three SNR points in one call (snr_point 0, 1, 2)."""
    H = hstd_for(CODE)
    B = 64
    frame0 = STEP * 4
    sig = [oracle.sigma_for_snr(s) for s in (1.0, 2.0, 3.0)]
    dec = _decoder(B)
    ctr = dec.mc_run(SEED, sig, B, frame0, T, static=True)
    for p, s in enumerate(sig):
        u, llr = dec.generate(SEED, p, s, frame0, B)
        _, want = _want(H, u, llr)
        np.testing.assert_array_equal(ctr[p], want, err_msg=f"point {p}")
    # the streaming schedule (ldpc_mc_run's default, bench's extra SNR points) agrees
    stream = dec.mc_run(SEED, sig, B, frame0, T)
    np.testing.assert_array_equal(stream, ctr)


def test_bench_3db_point_shape(gpu_available):
    """The bench's whole 3 dB point at its real shape: 262,144 frames of
    wimax_2304_0.5 streamed through 8,192 slots in ONE mc_run (supply order,
    tile_sub_stream_kernel, hand-off, split tail: `bench.py --point-snr 3.0`),
    at the default bench's frame offset -- counters equal to the static
    schedule's over the same frames (8 chunks of 32,768), and the frames the
    supply order puts first (heaviest syndromes: the likely failures) and last
    decoded by the oracle, frame for frame, equal to the static decoder's."""
    from ldpc_amd.device import Decoder, Graph
    code = "wimax_2304_0.5"
    H = hstd_for(code)
    g = Graph.cached(H)
    PF, slots, T = 262144, STEP // 4, 50
    base = (1 + 3 + 2) * STEP  # bench.py defaults: warmup 1, steps 3, two extra points
    sg = oracle.sigma_for_snr(3.0)
    dec = Decoder(g, slots)
    dec.profile(True)
    a = dec.mc_run(SEED, [sg], PF, base, T)
    p = dec.profile_read()
    dec.profile(False)
    order = dec.frame_order(SEED, 0, sg, base, PF)
    dec.close()
    assert p["tile"][1] == 1 and p["cn"][1] > 0, p  # the supply kernel, then the split tail
    big = Decoder(g, STEP)
    b = big.mc_run(SEED, [sg], PF, base, T, static=True)
    np.testing.assert_array_equal(a, b)
    assert a[0, 0] == PF and 0 < a[0, 1] < PF // 10  # FER a few per cent at 3 dB
    # spot check: the first and last 48 frames of the supply order
    for idx in (order[:48], order[-48:]):
        us, ls = [], []
        for i in idx:
            u, llr = big.generate(SEED, 0, sg, base + int(i), 1)
            us.append(u[0])
            ls.append(llr[0])
        llr = np.stack(ls)
        r = big.decode(llr, T)
        o = oracle.spa_decode(H, llr, T)
        np.testing.assert_array_equal(r.z, o["z"])
        np.testing.assert_array_equal(r.conv, o["conv"])
    big.close()
