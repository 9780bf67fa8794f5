"""The tile-resident decoder (tile_kernels.hip) against the per-iteration
CN/VN launches (LDPC_F_SPLIT) and the oracle.

Both paths do every fp64 operation of spa_decoder.py in the reference's order,
so their outputs -- hard bits, convergence iteration, Result, iterations,
posteriors, messages, normalized LLR and its per-iteration history -- must be
IDENTICAL bit for bit, not merely close.  The golden-vector and oracle tests
(test_gpu_parity.py) already run through the tile path for the codes it
serves (BCH, wimax_576_0.5); these add the direct A/B on harder inputs.
"""
import numpy as np
import pytest

import oracle
from conftest import hstd_for
from test_gpu_parity import _random_llr

pytestmark = pytest.mark.gpu


def _decoder(code, frames):
    from ldpc_amd.device import Decoder, Graph
    return Decoder(Graph.cached(hstd_for(code)), frames)


def _assert_identical(a, b):
    for key in ("z", "conv", "status", "iters", "post", "msgs", "nllr", "hist"):
        va, vb = getattr(a, key), getattr(b, key)
        if va is None and vb is None:
            continue
        np.testing.assert_array_equal(va, vb, err_msg=key)


def test_tile_path_is_the_one_launched(gpu_available):
    dec = _decoder("wimax_576_0.5", 64)
    llr = _random_llr(hstd_for("wimax_576_0.5"), 64, 1.0, seed=1)
    dec.profile(True)
    dec.decode(llr, 3)
    p = dec.profile_read()
    dec.profile(False)
    assert p["tile"][1] == 1 and p["cn"][1] == 0 and p["vn"][1] == 0, p


@pytest.mark.parametrize("snr,T,B", [(-1.0, 7, 130), (0.5, 30, 64), (1.5, 12, 200), (2.5, 50, 70), (4.0, 5, 64)])
def test_tile_bit_identical_to_split(gpu_available, snr, T, B):
    code = "wimax_576_0.5"
    llr = _random_llr(hstd_for(code), B, snr, seed=int(100 * snr) + 1000 + T)
    dec = _decoder(code, B)
    a = dec.decode(llr, T, nllr=True, post=True, hist=True, msgs=True)
    b = dec.decode(llr, T, nllr=True, post=True, hist=True, msgs=True, split=True)
    _assert_identical(a, b)


def test_tile_rare_rows_identical_and_match_oracle(gpu_available):
    """Exact zeros and tiny LLRs send rows down the |t| <= 1e-10 branch."""
    code = "wimax_576_0.5"
    H = hstd_for(code)
    rng = np.random.default_rng(17)
    llr = _random_llr(H, 96, 1.0, seed=9)
    llr[0, :] = 0.0
    llr[1, ::5] = 0.0
    llr[2, :] = 1e-13
    llr[3, :] = rng.choice([-1, 1], 576) * 60.0
    llr[70, ::3] = 0.0  # a second tile with rare rows
    for T in (1, 4):
        dec = _decoder(code, 96)
        a = dec.decode(llr, T, nllr=True, post=True, msgs=True)
        b = dec.decode(llr, T, nllr=True, post=True, msgs=True, split=True)
        _assert_identical(a, b)
        o = oracle.spa_decode(H, llr, T, nllr=True)
        np.testing.assert_array_equal(a.z, o["z"])
        np.testing.assert_array_equal(a.conv, o["conv"])


def test_tile_bch_identical_to_split(gpu_available):
    code = "BCH_7_4_1_strip"
    llr = _random_llr(hstd_for(code), 1000, 0.0, seed=4)
    llr[:50, ::2] = 0.0
    dec = _decoder(code, 1000)
    for T in (1, 3, 10):
        _assert_identical(dec.decode(llr, T, nllr=True, post=True, hist=True, msgs=True),
                          dec.decode(llr, T, nllr=True, post=True, hist=True, msgs=True, split=True))


def test_tile_mc_counters_equal_split(gpu_available):
    dec = _decoder("wimax_576_0.5", 1024)
    sig = [oracle.sigma_for_snr(s) for s in (0.0, 1.5, 3.0)]
    a = dec.mc_run(20260213, sig, 2048, 0, 20, nllr=True, static=True)
    b = dec.mc_run(20260213, sig, 2048, 0, 20, nllr=True, static=True, split=True)
    np.testing.assert_array_equal(a, b)


# --- sub-tile decoder (tile_sub.hip): the WiMAX 2304 codes, 16 or 8 frames per
# workgroup, lane groups sharing one wavefront's chunk of a check row.  The
# 16-frame form (wimax_2304_0.5) is the default; the 8-frame form (r3/4) is
# opt-in (LDPC_TILE_SUB=1, read by the library at every decode)


@pytest.fixture
def sub_tile(monkeypatch):
    monkeypatch.setenv("LDPC_TILE_SUB", "1")


def test_sub_tile_default_for_half_rate_opt_in_for_three_quarter(gpu_available, monkeypatch):
    from ldpc_amd import _lib
    monkeypatch.delenv("LDPC_TILE_SUB", raising=False)
    assert _lib.lib().ldpc_tile_kernel_name(_decoder("wimax_2304_0.5", 64).graph.handle) == b"tile_sub_kernel"
    assert _lib.lib().ldpc_tile_kernel_name(_decoder("wimax_2304_0.75A", 64).graph.handle) == b""
    monkeypatch.setenv("LDPC_TILE_SUB", "0")
    assert _lib.lib().ldpc_tile_kernel_name(_decoder("wimax_2304_0.5", 64).graph.handle) == b""


def test_sub_tile_is_the_one_launched(gpu_available, sub_tile):
    from ldpc_amd import _lib
    for code in ("wimax_2304_0.5", "wimax_2304_0.75A"):
        dec = _decoder(code, 64)
        assert _lib.lib().ldpc_tile_kernel_name(dec.graph.handle) == b"tile_sub_kernel"
        llr = _random_llr(hstd_for(code), 64, 1.0, seed=2)
        dec.profile(True)
        dec.decode(llr, 2)
        p = dec.profile_read()
        dec.profile(False)
        assert p["tile"][1] == 1 and p["cn"][1] == 0 and p["vn"][1] == 0, p


@pytest.mark.parametrize("code,snr,T,B", [("wimax_2304_0.5", 0.0, 4, 70), ("wimax_2304_0.5", 3.0, 25, 40),
                                          ("wimax_2304_0.75A", 2.0, 5, 64), ("wimax_2304_0.75B", 4.0, 8, 24)])
def test_sub_tile_bit_identical_to_split(gpu_available, sub_tile, code, snr, T, B):
    llr = _random_llr(hstd_for(code), B, snr, seed=int(100 * snr) + 2000 + T)
    dec = _decoder(code, B)
    a = dec.decode(llr, T, nllr=True, post=True, hist=True, msgs=True)
    b = dec.decode(llr, T, nllr=True, post=True, hist=True, msgs=True, split=True)
    _assert_identical(a, b)


def test_sub_tile_rare_rows_identical(gpu_available, sub_tile):
    code = "wimax_2304_0.5"
    H = hstd_for(code)
    llr = _random_llr(H, 80, 1.0, seed=19)
    llr[0, :] = 0.0
    llr[5, ::7] = 0.0
    llr[17, :] = 1e-13
    llr[66, ::3] = 0.0  # another 64-frame tile, another sub-tile
    dec = _decoder(code, 80)
    for T in (1, 3):
        _assert_identical(dec.decode(llr, T, nllr=True, post=True, msgs=True),
                          dec.decode(llr, T, nllr=True, post=True, msgs=True, split=True))


@pytest.mark.parametrize("snr,T,B", [(0.0, 4, 70), (3.0, 25, 40)])
def test_cn_row16_bit_identical_to_sub_tile(gpu_available, monkeypatch, snr, T, B):
    """The 16-wavefront x 40-edge cn_row_kernel shape (rows of wimax_2304_0.5;
    by default only from 64 tiles on, forced here) == the sub-tile decoder."""
    code = "wimax_2304_0.5"
    llr = _random_llr(hstd_for(code), B, snr, seed=int(100 * snr) + 3000 + T)
    llr[1, ::5] = 0.0  # a rare row (|t| <= 1e-10) for cn_rare_kernel
    dec = _decoder(code, B)
    a = dec.decode(llr, T, nllr=True, post=True, hist=True, msgs=True)
    monkeypatch.setenv("LDPC_CN_ROW16", "1")
    b = dec.decode(llr, T, nllr=True, post=True, hist=True, msgs=True, split=True)
    _assert_identical(a, b)
