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


@pytest.fixture(autouse=True)
def _tile_path_at_any_size(monkeypatch):
    """These tests exercise the tile kernels on small batches: keep the
    small-batch column-parallel path (LDPC_SMALL_COLS, test_gpu_smallcols.py)
    out of the way."""
    monkeypatch.setenv("LDPC_SMALL_COLS", "0")


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


# --- the WiMAX 2304 codes: the 8-frame sub-tile decoder (tile8.hip, the
# default: E in 8-frame blocks, DevGraph::ef = 8) and, with LDPC_TILE8=0 at
# graph creation, the older 16-frame sub-tile decoder (tile_sub.hip, r1/2 only)


def _fresh_decoder(code, frames, tile8=None, monkeypatch=None):
    """A decoder on a NEW graph (the layout is chosen at graph creation):
    tile8 True / False sets LDPC_TILE8=1 / 0 for it, None keeps the default."""
    from ldpc_amd.device import Decoder, Graph
    if tile8 is not None:
        monkeypatch.setenv("LDPC_TILE8", "1" if tile8 else "0")
    try:
        return Decoder(Graph(hstd_for(code)), frames)
    finally:
        if tile8 is not None:
            monkeypatch.delenv("LDPC_TILE8")


def _t8(code, frames, monkeypatch):
    """A decoder that runs tile8_kernel (wimax_2304_0.5 needs LDPC_TILE8=1)."""
    return _fresh_decoder(code, frames, tile8=True, monkeypatch=monkeypatch)


def test_tile8_default_for_three_quarter_codes(gpu_available, monkeypatch):
    from ldpc_amd import _lib
    name = lambda d: _lib.lib().ldpc_tile_kernel_name(d.graph.handle)  # noqa: E731
    for code in ("wimax_2304_0.75A", "wimax_2304_0.75B"):
        assert name(_decoder(code, 64)) == b"tile8_kernel", code
    assert name(_decoder("wimax_2304_0.5", 64)) == b"tile_sub_kernel"
    assert name(_decoder("wimax_576_0.5", 64)) == b"tile_kernel"
    assert name(_t8("wimax_2304_0.5", 64, monkeypatch)) == b"tile8_kernel"
    assert name(_fresh_decoder("wimax_2304_0.75A", 64, tile8=False, monkeypatch=monkeypatch)) == b""


def test_tile8_is_the_one_launched(gpu_available, monkeypatch):
    for code in ("wimax_2304_0.5", "wimax_2304_0.75A"):
        dec = _t8(code, 64, monkeypatch)
        llr = _random_llr(hstd_for(code), 64, 1.0, seed=2)
        dec.profile(True)
        dec.decode(llr, 2)
        p = dec.profile_read()
        dec.profile(False)
        assert p["tile"][1] == 1 and p["cn"][1] == 0 and p["vn"][1] == 0, p


@pytest.mark.parametrize("code,snr,T,B", [("wimax_2304_0.5", 0.0, 4, 70), ("wimax_2304_0.5", 3.0, 25, 40),
                                          ("wimax_2304_0.5", 1.0, 50, 64),
                                          ("wimax_2304_0.75A", 2.0, 5, 64), ("wimax_2304_0.75A", 1.0, 30, 72),
                                          ("wimax_2304_0.75B", 4.0, 8, 24),
                                          # saturated rows (config 4's 3.5 / 4 dB: tile8's P3 memo,
                                          # LDPC_T8_SATMEMO) against the split path's per-edge atanh
                                          ("wimax_2304_0.75A", 4.0, 50, 72), ("wimax_2304_0.75A", 3.5, 20, 64)])
def test_tile8_bit_identical_to_split(gpu_available, monkeypatch, code, snr, T, B):
    llr = _random_llr(hstd_for(code), B, snr, seed=int(100 * snr) + 2000 + T)
    dec = _t8(code, B, monkeypatch)
    a = dec.decode(llr, T, nllr=True, post=True, hist=True, msgs=True)
    b = dec.decode(llr, T, nllr=True, post=True, hist=True, msgs=True, split=True)
    _assert_identical(a, b)


@pytest.mark.parametrize("code", ["wimax_2304_0.5", "wimax_2304_0.75A"])
def test_tile8_identical_to_the_16_frame_layout(gpu_available, monkeypatch, code):
    """E in 8-frame blocks (tile8 + its split path) == the 64-frame layout
    (tile_sub_kernel or the split path on [tile][edge][64]), every output."""
    llr = _random_llr(hstd_for(code), 90, 1.5, seed=77)
    a = _t8(code, 90, monkeypatch).decode(llr, 12, nllr=True, post=True, hist=True, msgs=True)
    b = _fresh_decoder(code, 90, tile8=False, monkeypatch=monkeypatch).decode(
        llr, 12, nllr=True, post=True, hist=True, msgs=True)
    _assert_identical(a, b)


@pytest.mark.parametrize("code", ["wimax_2304_0.5", "wimax_2304_0.75A"])
def test_tile8_rare_rows_identical(gpu_available, monkeypatch, code):
    H = hstd_for(code)
    n = H.shape[1]
    llr = _random_llr(H, 80, 1.0, seed=19)
    llr[0, :] = 0.0
    llr[5, ::7] = 0.0
    llr[17, :] = 1e-13
    llr[66, ::3] = 0.0  # another 64-frame tile, another sub-tile
    llr[9, : n // 2] = 0.0
    dec = _t8(code, 80, monkeypatch)
    for T in (1, 3):
        _assert_identical(dec.decode(llr, T, nllr=True, post=True, msgs=True),
                          dec.decode(llr, T, nllr=True, post=True, msgs=True, split=True))


def test_sub_tile16_still_identical(gpu_available, monkeypatch):
    """The retained 16-frame sub-tile decoder (LDPC_TILE8=0) == its split path."""
    code = "wimax_2304_0.5"
    llr = _random_llr(hstd_for(code), 40, 3.0, seed=2025)
    dec = _fresh_decoder(code, 40, tile8=False, monkeypatch=monkeypatch)
    _assert_identical(dec.decode(llr, 25, nllr=True, post=True, hist=True, msgs=True),
                      dec.decode(llr, 25, nllr=True, post=True, hist=True, msgs=True, split=True))


@pytest.mark.parametrize("snr,T,B", [(0.0, 4, 70), (3.0, 25, 40)])
def test_cn_row16_bit_identical_to_sub_tile(gpu_available, monkeypatch, snr, T, B):
    """The 16-wavefront x 40-edge cn_row_kernel shape (rows of wimax_2304_0.5;
    by default only from 64 tiles on, forced here) == the tile decoder."""
    code = "wimax_2304_0.5"
    llr = _random_llr(hstd_for(code), B, snr, seed=int(100 * snr) + 3000 + T)
    llr[1, ::5] = 0.0  # a rare row (|t| <= 1e-10) for cn_rare_kernel
    dec = _decoder(code, B)
    a = dec.decode(llr, T, nllr=True, post=True, hist=True, msgs=True)
    monkeypatch.setenv("LDPC_CN_ROW16", "1")
    monkeypatch.setenv("LDPC_CN_SUB", "0")  # cn_sub_kernel would take these small batches
    b = dec.decode(llr, T, nllr=True, post=True, hist=True, msgs=True, split=True)
    _assert_identical(a, b)


@pytest.mark.parametrize("code,snr,T,B", [("wimax_2304_0.5", 0.0, 4, 70), ("wimax_2304_0.5", 3.0, 25, 40),
                                          ("wimax_2304_0.5", 1.0, 1, 64),
                                          ("wimax_2304_0.75A", 2.0, 6, 72), ("wimax_2304_0.75B", 3.5, 10, 64)])
def test_cn_sub_bit_identical_to_cn_kernel(gpu_available, monkeypatch, code, snr, T, B):
    """cn_sub_kernel (16-frame sub-tiles, t in registers, one tanh per edge:
    the split CN of the long-row codes up to LDPC_CN_SUB tiles) == cn_kernel
    (one wavefront per row, two tanh per edge), every output, with rare rows
    (exact zeros, tiny LLRs: the sub-tile's frames go to cn_rare_kernel) and
    ragged batches."""
    H = hstd_for(code)
    llr = _random_llr(H, B, snr, seed=int(100 * snr) + 5000 + T)
    llr[1, ::5] = 0.0
    llr[3, :] = 1e-13
    llr[B - 1, ::9] = 0.0  # a rare row in the last (possibly partial) sub-tile
    dec = _decoder(code, B)
    monkeypatch.setenv("LDPC_SMALL_COLS", "0")  # the split path with the per-tile vn_kernel
    a = dec.decode(llr, T, nllr=True, post=True, hist=True, msgs=True, split=True)
    monkeypatch.setenv("LDPC_CN_SUB", "0")
    b = dec.decode(llr, T, nllr=True, post=True, hist=True, msgs=True, split=True)
    _assert_identical(a, b)


def test_cn_sub_stream_counters(gpu_available, monkeypatch):
    """The streaming split loop (fresh frames, refills, compaction, the
    column-parallel tail VN) with cn_sub_kernel == with cn_kernel."""
    import oracle as _o
    code = "wimax_2304_0.5"
    dec = _decoder(code, 256)
    sig = [_o.sigma_for_snr(s) for s in (2.5, 3.0)]
    a = dec.mc_run(20260213, sig, 900, 33, 20, nllr=True, split=True)
    monkeypatch.setenv("LDPC_CN_SUB", "0")
    b = dec.mc_run(20260213, sig, 900, 33, 20, nllr=True, split=True)
    np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("code,lo,hi", [("wimax_576_0.5", 0.011, 0.015),     # tile_kernel
                                        ("wimax_2304_0.5", 0.5, 0.7),         # tile_sub_kernel<4>
                                        ("wimax_2304_0.75A", 0.85, 1.05)])    # tile8_kernel
def test_subnormal_column_sums_identical(gpu_available, code, lo, hi):
    """The tile decoders add E_new into the LDS column sums with ds_add_f64
    (LDPC_*_LDSADD); the split path adds with v_add_f64 in vn_kernel.  LLR
    magnitudes chosen so the row products underflow: ~28-50 % of the messages
    are subnormal (checked below), so a flushing add would show."""
    H = hstd_for(code)
    rng = np.random.default_rng(5)
    B = 70
    llr = rng.uniform(lo, hi, (B, H.shape[1])) * rng.choice([-1.0, 1.0], (B, H.shape[1]))
    dec = _decoder(code, B)
    a = dec.decode(llr, 2, nllr=True, post=True, hist=True, msgs=True)
    b = dec.decode(llr, 2, nllr=True, post=True, hist=True, msgs=True, split=True)
    sub = (a.msgs != 0) & (np.abs(a.msgs) < np.finfo(np.float64).tiny)
    assert sub.mean() > 0.2, sub.mean()
    _assert_identical(a, b)
