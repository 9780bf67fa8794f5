"""The reference's rare-row branch (|t| <= 1e-10: the product of the OTHER
tanh values, spa_decoder.py:159-164) through the STREAMING Monte-Carlo kernels,
against the oracle.

The tile decoders park a rare row's t in scratch and, since round 5, alternate
two buffers between consecutive rare rows (a single buffer raced: b946036).
The static routes are pinned by tests/test_gpu_decoders.py
test_2304_rare_rows; this file drives the same branch through the streaming
kernels (refilled slots next to old ones) and through the split tail they hand
off to (cn_sub_kernel -> cn_rare_kernel).

Rare rows come from the frame source's test-only erasures (LDPC_F_TEST_ZERO,
frame_source.h test_zero_llr): frames with F % 4 == 1 get a channel LLR of
exactly 0.0 on one identity column and one information column.  An identity
column has degree 1 in H_std = [A | I], so its M = (0 + E) - E is 0 on every
iteration, and its row is rare on every pass of that frame -- in the stream
kernel and, if the frame is still running at hand-off, in the tail.
"""
import numpy as np
import pytest

import oracle
from conftest import hstd_for

pytestmark = pytest.mark.gpu

SEED = 20260613


def zero_cols(F, k, m):
    """The erasure predicate of frame_source.h test_zero_llr, restated."""
    if F % 4 != 1:
        return []
    return [k + (131 * F + 7) % m, (37 * F + 3) % k]


def _decoder(code, frames):
    from ldpc_amd.device import Decoder, Graph
    return Decoder(Graph.cached(hstd_for(code)), frames)


@pytest.mark.parametrize("code", ["wimax_576_0.5", "wimax_2304_0.5", "wimax_2304_0.75A"])
def test_generator_test_zero_predicate(gpu_available, code):
    """The flag changes exactly the predicted LLRs, to exactly 0.0, and nothing else."""
    H = hstd_for(code)
    m, n = H.shape
    k = n - m
    dec = _decoder(code, 128)
    sg = oracle.sigma_for_snr(2.0)
    u0, l0 = dec.generate(SEED, 1, sg, 4001, 128)
    u1, l1 = dec.generate(SEED, 1, sg, 4001, 128, test_zero=True)
    np.testing.assert_array_equal(u0, u1)
    want = l0.copy()
    for f in range(128):
        for j in zero_cols(4001 + f, k, m):
            want[f, j] = 0.0
    np.testing.assert_array_equal(l1, want)
    assert (l1 == 0.0).sum() == 2 * sum(1 for f in range(128) if (4001 + f) % 4 == 1)


# (code, snr, expect_tail): 192 frames through 64 slots at T = 50, so refilled
# slots decode erased frames next to slots still holding older ones
CASES = [
    ("wimax_2304_0.5", 2.5, True),    # tile_sub_stream_kernel -> hand-off -> cn_sub + cn_rare tail
    ("wimax_2304_0.5", 3.0, True),
    ("wimax_2304_0.75A", 2.5, True),  # tile8_stream_kernel -> hand-off -> cn_sub + cn_rare tail
    ("wimax_576_0.5", 2.0, False),    # tile_stream_kernel (drains in-kernel, no hand-off)
]


@pytest.mark.parametrize("code,snr,expect_tail", CASES)
def test_stream_rare_rows_match_oracle(gpu_available, code, snr, expect_tail):
    H = hstd_for(code)
    m, n = H.shape
    k = n - m
    cap, frames, T, frame0 = 64, 192, 50, 9001
    sg = oracle.sigma_for_snr(snr)
    dec = _decoder(code, cap)
    dec.rare_rows()  # reset the running totals
    dec.profile(True)
    ctr = dec.mc_run(SEED, [sg], frames, frame0, T, nllr=True, test_zero=True)
    p = dec.profile_read()
    dec.profile(False)
    split_rare, tile_rare = dec.rare_rows()
    assert p["tile"][1] == 1, p  # one streaming tile-kernel launch
    assert tile_rare > 0, (split_rare, tile_rare)  # the streaming kernel took rare rows in-kernel
    if expect_tail:
        assert p["cn"][1] > 0 and p["vn_cols"][1] > 0, p  # the split tail ran ...
        assert split_rare > 0, (split_rare, tile_rare)  # ... and sent rare rows to cn_rare_kernel
    u, llr = _decoder(code, frames).generate(SEED, 0, sg, frame0, frames, test_zero=True)
    assert (llr == 0.0).sum() >= frames // 4 * 2
    o = oracle.spa_decode(H, llr, T, nllr=True)
    want = oracle.main_counters(u, o["z"], o["status"], o["conv"],
                                nllr_cnt=np.rint(o["nllr"] * k).astype(np.int64), iters=o["iters"])
    np.testing.assert_array_equal(ctr[0], want)
    # the same frames decoded by decode() (static tile decoder), frame by frame
    r = _decoder(code, frames).decode(llr, T, nllr=True)
    np.testing.assert_array_equal(r.z, o["z"])
    np.testing.assert_array_equal(r.conv, o["conv"])
    np.testing.assert_array_equal(r.status, o["status"])
    # and the static Monte-Carlo schedule and the split streaming loop agree
    np.testing.assert_array_equal(dec.mc_run(SEED, [sg], frames, frame0, T, nllr=True, test_zero=True,
                                             static=True), ctr)
    np.testing.assert_array_equal(dec.mc_run(SEED, [sg], frames, frame0, T, nllr=True, test_zero=True,
                                             split=True), ctr)
