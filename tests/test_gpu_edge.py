"""The few-frame decode path (edge_kernels.hip: lanes over a row's / column's
edges, frame after frame; ldpc_api.cpp small_batch_edge): main.py's one-frame
decode() calls.  Its outputs -- hard bits, convergence iteration, Result,
iterations, posteriors, messages, normalized LLR and its history -- must be
identical bit for bit to the frame-per-lane split path's (cn_kernel +
cn_rare_kernel with the column-parallel VN, LDPC_EDGE_FRAMES=0) and to the
per-tile vn_kernel's, match the oracle, and be the path that runs."""
import numpy as np
import pytest

import oracle
from conftest import hstd_for, load_golden
from test_gpu_parity import _random_llr
from test_gpu_tile import _assert_identical

pytestmark = pytest.mark.gpu


def _decoder(code, frames):
    from ldpc_amd.device import Decoder, Graph
    return Decoder(Graph.cached(hstd_for(code)), frames)


def _three_ways(dec, llr, T, monkeypatch):
    a = dec.decode(llr, T, nllr=True, post=True, hist=True, msgs=True)  # the edge path
    monkeypatch.setenv("LDPC_EDGE_FRAMES", "0")
    b = dec.decode(llr, T, nllr=True, post=True, hist=True, msgs=True)  # frame per lane, column-parallel VN
    monkeypatch.setenv("LDPC_SMALL_COLS", "0")
    c = dec.decode(llr, T, nllr=True, post=True, hist=True, msgs=True, split=True)  # per-tile vn_kernel
    monkeypatch.delenv("LDPC_EDGE_FRAMES")
    monkeypatch.delenv("LDPC_SMALL_COLS")
    return a, b, c


@pytest.mark.parametrize("code,snr,T,B", [
    ("wimax_2304_0.5", 1.0, 12, 1), ("wimax_2304_0.5", 2.5, 30, 3), ("wimax_2304_0.5", 3.0, 50, 8),
    ("wimax_2304_0.75A", 2.0, 10, 1), ("wimax_2304_0.75A", 3.5, 25, 5), ("wimax_2304_0.75B", 2.0, 8, 2)])
def test_edge_path_identical_to_frame_per_lane(gpu_available, monkeypatch, code, snr, T, B):
    llr = _random_llr(hstd_for(code), B, snr, seed=int(10 * snr) + 17 * B + T)
    dec = _decoder(code, 64)
    a, b, c = _three_ways(dec, llr, T, monkeypatch)
    _assert_identical(a, b)
    _assert_identical(a, c)


def test_edge_rare_rows_identical_and_match_oracle(gpu_available, monkeypatch):
    """Exact zeros and tiny LLRs send rows down the |t| <= 1e-10 branch (the
    product of the others, formed inside cn_edge_kernel)."""
    code = "wimax_2304_0.5"
    H = hstd_for(code)
    rng = np.random.default_rng(23)
    llr = _random_llr(H, 6, 1.5, seed=19)
    llr[0, :] = 0.0
    llr[1, ::7] = 0.0
    llr[2, :] = 1e-13
    llr[3, :] = rng.choice([-1, 1], H.shape[1]) * 60.0
    llr[4, 5] = 0.0  # one zero: a single rare edge in a few rows
    dec = _decoder(code, 64)
    for T in (1, 3):
        a, b, c = _three_ways(dec, llr, T, monkeypatch)
        _assert_identical(a, b)
        _assert_identical(a, c)
        o = oracle.spa_decode(H, llr, T, nllr=True)
        np.testing.assert_array_equal(a.z, o["z"])
        np.testing.assert_array_equal(a.conv, o["conv"])


def test_edge_path_matches_reference_golden(gpu_available):
    """Frames the reference itself decoded (wimax_2304_0.5, T=50 at 1 and 3 dB),
    one decode() call per frame as main.py makes them."""
    g = load_golden("w2304_T50")
    H = hstd_for(str(g["code"]))
    dec = _decoder(str(g["code"]), 64)
    T = int(g["T"])
    for i in range(0, len(g["ch"]), 5):
        r = dec.decode(g["ch"][i:i + 1], T, nllr=bool(g["nllr_on"]))
        np.testing.assert_array_equal(r.z[0], g["z"][i])
        assert int(r.conv[0]) == int(g["conv"][i])
        assert bool(r.status[0] == 0) == bool(g["ok"][i])
    del H


def test_edge_path_is_the_one_launched(gpu_available, monkeypatch):
    """A one-frame call and a 9-frame call (both <= LDPC_EDGE_FRAMES, 32 for
    the 2304 codes) run cn_edge_kernel + vn_edge_kernel and nothing else
    (the exact cut-overs: tests/test_gpu_decoders.py test_cutover_thresholds)."""
    dec = _decoder("wimax_2304_0.5", 64)
    llr = _random_llr(hstd_for("wimax_2304_0.5"), 9, 2.0, seed=5)
    for B in (1, 9):
        dec.profile(True)
        dec.decode(llr[:B], 4)
        p = dec.profile_read()
        dec.profile(False)
        assert p["cn_edge"][1] == 4 and p["vn_edge"][1] == 4, p
        assert p["tile"][1] == 0 and p["cn"][1] == 0 and p["vn"][1] == 0 and p["vn_cols"][1] == 0, p
    # both calls agree with the frame-per-lane path on their frames
    monkeypatch.setenv("LDPC_EDGE_FRAMES", "0")
    a = dec.decode(llr, 4, post=True)
    monkeypatch.delenv("LDPC_EDGE_FRAMES")
    b = dec.decode(llr, 4, post=True)
    np.testing.assert_array_equal(a.post, b.post)
