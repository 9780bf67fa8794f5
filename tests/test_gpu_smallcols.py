"""Small decode batches of the long-row codes above the few-frame edge path's
limit (LDPC_EDGE_FRAMES, 32 frames) and up to LDPC_SMALL_COLS tiles run the
split CN with the column-parallel VN (vn_cols_kernel + tail_exit_kernel<true>;
ldpc_api.cpp small_batch_cols).  Its outputs -- hard bits, convergence
iteration, Result, iterations, posteriors, messages, normalized LLR and its
per-iteration history -- must be identical bit for bit to the per-tile
vn_kernel's (the split path with LDPC_SMALL_COLS=0) and to the sub-tile
decoders', and it must be the path that runs (profile kinds cn + vn_cols).
The one-frame calls of main.py take the edge path instead
(tests/test_gpu_edge.py)."""
import numpy as np
import pytest

from conftest import hstd_for
from test_gpu_parity import _random_llr
from test_gpu_tile import _assert_identical

pytestmark = pytest.mark.gpu


def _decoder(code, frames):
    from ldpc_amd.device import Decoder, Graph
    return Decoder(Graph.cached(hstd_for(code)), frames)


@pytest.mark.parametrize("code,snr,T,B", [
    ("wimax_2304_0.5", 1.0, 6, 1), ("wimax_2304_0.5", 2.5, 20, 70), ("wimax_2304_0.5", 3.0, 50, 64),
    ("wimax_2304_0.75A", 2.0, 8, 5), ("wimax_2304_0.75A", 3.5, 30, 130)])
def test_small_batch_cols_identical_to_vn_kernel_and_tile(gpu_available, monkeypatch, code, snr, T, B):
    llr = _random_llr(hstd_for(code), B, snr, seed=int(10 * snr) + 31 * B + T)
    dec = _decoder(code, max(B, 64))
    monkeypatch.setenv("LDPC_EDGE_FRAMES", "0")  # B <= 32 would take the edge path
    dec.profile(True)
    a = dec.decode(llr, T, nllr=True, post=True, hist=True, msgs=True)
    p = dec.profile_read()
    dec.profile(False)
    monkeypatch.delenv("LDPC_EDGE_FRAMES")
    # the split CN + column-parallel VN ran, nothing else
    assert p["cn"][1] > 0 and p["vn_cols"][1] > 0, p
    assert p["tile"][1] == 0 and p["vn"][1] == 0 and p["cn_edge"][1] == 0 and p["vn_edge"][1] == 0, p
    monkeypatch.setenv("LDPC_SMALL_COLS", "0")
    b = dec.decode(llr, T, nllr=True, post=True, hist=True, msgs=True, split=True)  # per-tile vn_kernel
    c = dec.decode(llr, T, nllr=True, post=True, hist=True, msgs=True)  # the sub-tile decoder
    _assert_identical(a, b)
    _assert_identical(a, c)


def test_dropin_decode_uses_small_batch_path(gpu_available):
    """SPA_Decoder.decode (one frame, 64 slots) takes the few-frame edge path."""
    dec = _decoder("wimax_2304_0.5", 64)
    llr = _random_llr(hstd_for("wimax_2304_0.5"), 1, 2.0, seed=5)
    dec.profile(True)
    dec.decode(llr, 10)
    p = dec.profile_read()
    dec.profile(False)
    assert p["cn_edge"][1] > 0 and p["vn_edge"][1] > 0, p
    assert p["tile"][1] == 0 and p["cn"][1] == 0 and p["vn"][1] == 0 and p["vn_cols"][1] == 0, p
