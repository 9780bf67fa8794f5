"""Every production decoder against the reference's own vectors and the oracle.

ldpc_decode_f64 picks one of five decoders per call (ldpc_api.cpp
run_iterations): the few-frame edge path (cn_edge_kernel + vn_edge_kernel,
batches up to LDPC_EDGE_FRAMES), the split CN + column-parallel VN
(vn_cols_kernel, up to LDPC_SMALL_COLS tiles of the long-row codes), the split
CN + per-tile vn_kernel, and the tile-resident decoders -- tile_kernel (64
frames: BCH, wimax_576_0.5), tile_sub_kernel<4> (16 frames: wimax_2304_0.5,
the headline) and tile8_kernel (8 frames: the r3/4 codes by default,
wimax_2304_0.5 when its graph is created with LDPC_TILE8=1).  The golden sets
are small (<= 32 frames for the 2304 codes), so the default route sends them
all down the edge path; here each set is FORCED through every decoder that
can serve its code, the profile counters prove which kernels ran, and the
outputs are held to the same bar as tests/test_gpu_parity.py: z, conv,
Result, iterations and nllr exact; L and E within 1e-5 relative (or the
oracle-measured conditioning slack on saturated frames).

Then tile8_kernel -- which had no direct oracle check -- on wimax_2304_0.75A
and 0.75B at T=50 over config 4's sweep (1, 2, 3, 4 dB; 4 dB is the
reference's FER-1.0 cliff), 72 frames = one full tile + one
ragged one (8 live frames: one live 8-frame sub-tile, seven empty).
Reference: python_ldpc_app/spa_decoder.py:63-280.
"""
import numpy as np
import pytest

import oracle
from conftest import GOLDEN_SETS, assert_llr_close, hstd_for, load_golden
from test_gpu_parity import _random_llr

pytestmark = pytest.mark.gpu

# route -> (environment, decode(split=...), kinds that must run, kinds that must not)
_ALL = ("cn", "vn", "tile", "cn_edge", "vn_edge", "vn_cols")
ROUTES = {
    # LDPC_EDGE_FRAMES large: every set, whatever its frame count, on the edge path
    "edge": ({"LDPC_EDGE_FRAMES": "100000"}, False, ("cn_edge", "vn_edge")),
    # frame per lane, column-parallel VN at any tile count (long-row codes only)
    "cols": ({"LDPC_EDGE_FRAMES": "0", "LDPC_SMALL_COLS": "100000"}, False, ("cn", "vn_cols")),
    # frame per lane, per-tile vn_kernel
    "split": ({"LDPC_SMALL_COLS": "0"}, True, ("cn", "vn")),
    # the tile-resident decoder of the graph (LDPC_SMALL_COLS=0 keeps both small-batch paths away)
    "tile": ({"LDPC_SMALL_COLS": "0"}, False, ("tile",)),
}
LONG = ("wimax_2304_0.5", "wimax_2304_0.75A", "wimax_2304_0.75B")


def _routes_for(code):
    """(route, graph layout) pairs that serve `code`.  layout: None = the
    default graph, 8 = created with LDPC_TILE8=1 (E in 8-frame blocks, tile8),
    64 = LDPC_TILE8=0 (E in 64-frame blocks)."""
    out = [("edge", None), ("split", None), ("tile", None)]
    if code in LONG:
        out.append(("cols", None))
    if code == "wimax_2304_0.5":  # the headline code also through tile8 (row and pair form) and its 8-frame split path
        out += [("tile", 8), ("split", 8), ("tile", "8p")]
    if code in ("wimax_2304_0.75A", "wimax_2304_0.75B"):  # the r3/4 codes in the 64-frame layout
        out += [("split", 64), ("cols", 64)]
    return out


def _tile_name(code, layout):
    if code in ("BCH_7_4_1_strip", "wimax_576_0.5"):
        return "tile_kernel"
    if code == "wimax_2304_0.5" and layout not in (8, "8p"):
        return "tile_sub_kernel"
    return "tile8_kernel:pair" if layout == "8p" else "tile8_kernel"


_GRAPHS = {}


def _graph(code, layout, monkeypatch):
    from ldpc_amd.device import Graph
    key = (code, layout)
    if key not in _GRAPHS:
        if layout is not None:
            monkeypatch.setenv("LDPC_TILE8", "0" if layout == 64 else "1")
        if layout == "8p":  # tile8's pair form (two rows per wavefront)
            monkeypatch.setenv("LDPC_T8_PAIR", "1")
        try:
            _GRAPHS[key] = Graph(hstd_for(code))
        finally:
            if layout is not None:
                monkeypatch.delenv("LDPC_TILE8")
            if layout == "8p":
                monkeypatch.delenv("LDPC_T8_PAIR")
    return _GRAPHS[key]


def _run_route(code, layout, route, llr, T, monkeypatch, **kw):
    """Decode through one route; assert from the profile that it ran and
    nothing else did.  -> DecodeResult."""
    from ldpc_amd import _lib
    from ldpc_amd.device import Decoder
    env, split, must = ROUTES[route]
    g = _graph(code, layout, monkeypatch)
    dec = Decoder(g, len(llr))
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    try:
        dec.profile(True)
        r = dec.decode(llr, T, split=split, **kw)
        p = dec.profile_read()
        dec.profile(False)
    finally:
        for k in env:
            monkeypatch.delenv(k)
    for kind in _ALL:
        ran = p[kind][1] > 0
        assert ran == (kind in must), (route, layout, kind, p)
    if route == "tile":
        assert p["tile"][1] == 1, p  # one launch: the whole batch, every iteration
        assert _lib.lib().ldpc_tile_kernel_name(g.handle).decode() == _tile_name(code, layout)
    dec.close()
    return r


_SLACK = {}


def _slack(set_name, g):
    if set_name not in _SLACK:
        _SLACK[set_name] = oracle.conditioning_slack(hstd_for(str(g["code"])), g["ch"], int(g["T"]),
                                                     nllr=bool(g["nllr_on"]))
    return _SLACK[set_name]


_CASES = [(s, r, lay) for s in GOLDEN_SETS for (r, lay) in _routes_for(str(load_golden(s)["code"]))]


@pytest.mark.parametrize("set_name,route,layout", _CASES,
                         ids=[f"{s}-{r}{'' if l is None else l}" for s, r, l in _CASES])
def test_golden_through_every_decoder(gpu_available, monkeypatch, set_name, route, layout):
    g = load_golden(set_name)
    code = str(g["code"])
    nl = bool(g["nllr_on"])
    T = int(g["T"])
    r = _run_route(code, layout, route, g["ch"], T, monkeypatch, nllr=nl, post=True, hist=nl, msgs=True)
    np.testing.assert_array_equal(r.z, g["z"], err_msg="hard decisions")
    np.testing.assert_array_equal(r.conv, g["conv"], err_msg="convergence_iteration")
    np.testing.assert_array_equal(r.status == 0, g["ok"], err_msg="Result")
    np.testing.assert_array_equal(r.iters, np.where(g["conv"] >= 0, g["conv"] + 1, T))
    if nl:
        np.testing.assert_array_equal(r.nllr, g["nllr"], err_msg="normalized LLR")
    es = int(g["e_stride"])
    try:  # plain 1e-5 first; the measured one-ulp slack only where that fails (saturated frames)
        assert_llr_close(r.post, g["L"], "posterior L")
        assert_llr_close(r.msgs[:, ::es], g["E"], "messages E")
    except AssertionError:
        sl_L, sl_E = _slack(set_name, g)
        assert_llr_close(r.post, g["L"], "posterior L", slack=sl_L)
        assert_llr_close(r.msgs[:, ::es], g["E"], "messages E", slack=sl_E[:, ::es])


_SWEEP = [(c, s) for c in ("wimax_2304_0.75A", "wimax_2304_0.75B") for s in (1.0, 2.0, 3.0, 4.0)]


@pytest.mark.parametrize("code,snr", _SWEEP, ids=[f"{c}-{s}dB" for c, s in _SWEEP])
def test_tile8_matches_oracle_config4_sweep(gpu_available, monkeypatch, code, snr):
    """tile8_kernel (the r3/4 codes' default decoder) vs the oracle at T=50."""
    H = hstd_for(code)
    T, B = 50, 72
    llr = _random_llr(H, B, snr, seed=4000 + int(10 * snr) + (0 if code.endswith("A") else 7))
    r = _run_route(code, None, "tile", llr, T, monkeypatch, nllr=True, post=True, msgs=True)
    o = oracle.spa_decode(H, llr, T, nllr=True, want_E=True)
    for key in ("z", "conv", "status", "iters", "nllr"):
        np.testing.assert_array_equal(r[key], o[key], err_msg=key)
    try:
        assert_llr_close(r.post, o["post"], "posterior L")
        assert_llr_close(r.msgs, o["msgs"], "messages E")
    except AssertionError:
        sl_L, sl_E = oracle.conditioning_slack(H, llr, T, nllr=True)
        assert_llr_close(r.post, o["post"], "posterior L", slack=sl_L)
        assert_llr_close(r.msgs, o["msgs"], "messages E", slack=sl_E)
    if snr == 4.0 and code.endswith("A"):
        assert (r.status == 1).mean() > 0.9  # the reference's own cliff (golden w2304A_T3_4dB)


_PAIR = [(s, n, "8p") for s in (1.0, 2.0, 3.0) for n in (72,)] + [(2.0, 130, "8p")]


@pytest.mark.parametrize("snr,B,layout", _PAIR, ids=[f"{l}-{s}dB-{n}" for s, n, l in _PAIR])
def test_tile8_pair_matches_oracle(gpu_available, monkeypatch, snr, B, layout):
    """tile8's pair form (two rows per wavefront, wimax_2304_0.5) vs the oracle
    at T=50: 72 frames (one full tile + one live 8-frame sub-tile) and 130
    (two full tiles + a 2-frame sub-tile)."""
    code = "wimax_2304_0.5"
    H = hstd_for(code)
    T = 50
    llr = _random_llr(H, B, snr, seed=5100 + int(10 * snr) + B)
    r = _run_route(code, layout, "tile", llr, T, monkeypatch, nllr=True, post=True, msgs=True)
    o = oracle.spa_decode(H, llr, T, nllr=True, want_E=True)
    for key in ("z", "conv", "status", "iters", "nllr"):
        np.testing.assert_array_equal(r[key], o[key], err_msg=key)
    try:
        assert_llr_close(r.post, o["post"], "posterior L")
        assert_llr_close(r.msgs, o["msgs"], "messages E")
    except AssertionError:
        sl_L, sl_E = oracle.conditioning_slack(H, llr, T, nllr=True)
        assert_llr_close(r.post, o["post"], "posterior L", slack=sl_L)
        assert_llr_close(r.msgs, o["msgs"], "messages E", slack=sl_E)


_RARE_ROUTES = [("tile", "8p"), ("tile", 8), ("tile", None), ("split", None), ("edge", None)]


@pytest.mark.parametrize("route,layout", _RARE_ROUTES, ids=[f"{r}{'' if l is None else l}" for r, l in _RARE_ROUTES])
def test_2304_rare_rows(gpu_available, monkeypatch, route, layout):
    """The rare path (|t| <= 1e-10: the product of the others,
    spa_decoder.py:159-164) of the wimax_2304_0.5 decoders -- tile8's pair
    form above all (a pair's two rows in one wavefront, either one tiny):
    frames with exact-zero channel LLRs on 1-4 columns, vs the oracle, T = 5."""
    code = "wimax_2304_0.5"
    H = hstd_for(code)
    B, T = 24, 5
    llr = _random_llr(H, B, 2.0, seed=77)
    rng = np.random.default_rng(78)
    for f in range(B):
        llr[f, rng.choice(H.shape[1], size=1 + f % 4, replace=False)] = 0.0
    r = _run_route(code, layout, route, llr, T, monkeypatch, nllr=True, post=True, msgs=True)
    o = oracle.spa_decode(H, llr, T, nllr=True, want_E=True)
    bad = np.nonzero((r.z != o["z"]).any(axis=1))[0]
    assert bad.size == 0, (bad, [np.nonzero(r.z[f] != o["z"][f])[0] for f in bad],
                           [np.nonzero(llr[f] == 0.0)[0] for f in bad])
    for key in ("z", "conv", "status", "iters", "nllr"):
        np.testing.assert_array_equal(r[key], o[key], err_msg=key)
    try:
        assert_llr_close(r.post, o["post"], "posterior L")
        assert_llr_close(r.msgs, o["msgs"], "messages E")
    except AssertionError:
        sl_L, sl_E = oracle.conditioning_slack(H, llr, T, nllr=True)
        assert_llr_close(r.post, o["post"], "posterior L", slack=sl_L)
        assert_llr_close(r.msgs, o["msgs"], "messages E", slack=sl_E)


def test_cutover_thresholds(gpu_available, monkeypatch):
    """The default batch-size cut-overs (ldpc_api.cpp small_batch_edge /
    small_batch_cols): 32 frames of a 2304 code run the edge path and 33 the
    split CN + column-parallel VN; wimax_576_0.5 (a 64-frame tile_kernel code)
    runs the edge path up to 4 frames and tile_kernel from 5."""
    from ldpc_amd.device import Decoder, Graph
    for code, lim, above in (("wimax_2304_0.5", 32, ("cn", "vn_cols")), ("wimax_576_0.5", 4, ("tile",))):
        dec = Decoder(Graph.cached(hstd_for(code)), 64)
        llr = _random_llr(hstd_for(code), lim + 1, 2.0, seed=lim)
        for B, must in ((lim, ("cn_edge", "vn_edge")), (lim + 1, above)):
            dec.profile(True)
            dec.decode(llr[:B], 3)
            p = dec.profile_read()
            dec.profile(False)
            for kind in _ALL:
                assert (p[kind][1] > 0) == (kind in must), (code, B, kind, p)
