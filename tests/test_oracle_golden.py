"""The CPU oracle (oracle/spa_oracle.c) against the reference's own outputs.

tests/golden/*.npz were produced by running python_ldpc_app/spa_decoder.py
itself (tests/golden/gen_golden.py).  This pins the oracle before anything is
compared against it: hard decisions, convergence iteration and Result must be
identical; final LLRs and messages within 1e-5 relative (the only allowed
difference is the ulp-level tanh/atanh of numpy's SVML vs glibc).
"""
import numpy as np
import pytest

import oracle
from conftest import GOLDEN_SETS, assert_llr_close, hstd_for, load_golden, max_rel

SETS = [s for s in GOLDEN_SETS]


@pytest.mark.parametrize("set_name", SETS)
def test_oracle_matches_reference(set_name):
    g = load_golden(set_name)
    H = hstd_for(str(g["code"]))
    r = oracle.spa_decode(H, g["ch"], int(g["T"]), nllr=bool(g["nllr_on"]), want_E=True)
    sl_L, sl_E = oracle.conditioning_slack(H, g["ch"], int(g["T"]), nllr=bool(g["nllr_on"]))
    sl_E = sl_E[:, :: int(g["e_stride"])]
    np.testing.assert_array_equal(r["z"], g["z"], err_msg="hard decisions")
    np.testing.assert_array_equal(r["conv"], g["conv"], err_msg="convergence_iteration")
    np.testing.assert_array_equal(r["status"] == 0, g["ok"], err_msg="Result")
    assert_llr_close(r["post"], g["L"], "posterior L", slack=sl_L)
    E = r["msgs"][:, :: int(g["e_stride"])]
    assert_llr_close(E, g["E"], "messages E", slack=sl_E)
    if bool(g["nllr_on"]):
        np.testing.assert_array_equal(r["nllr"], g["nllr"], err_msg="normalized LLR")
    # well-conditioned frames agree to the ulp level, far inside 1e-5
    well = (sl_L / np.maximum(np.abs(g["L"]), 1e-300)).max(axis=1) < 1e-6
    assert max_rel(r["post"][well], g["L"][well]) < 1e-7


def test_saturated_frames_are_few_and_flagged():
    """Only the deliberately saturated edge fixtures need conditioning slack."""
    for set_name in ("w576_T5", "w576_T50", "w2304_T3", "bch_T10"):
        g = load_golden(set_name)
        H = hstd_for(str(g["code"]))
        sl_L, _ = oracle.conditioning_slack(H, g["ch"], int(g["T"]))
        assert (sl_L <= 1e-5 * np.maximum(np.abs(g["L"]), 1e-3)).all(), set_name


def test_golden_sets_cover_rare_branches():
    """The edge fixtures must actually exercise |t|<=1e-10 and the clips."""
    g = load_golden("bch_edge_T1")
    assert (g["ch"] == 0.0).any() and (np.abs(g["ch"]) > 35.0).any()
    g = load_golden("w576_edge")
    assert (g["ch"] == 0.0).any() and (np.abs(g["ch"]) > 35.0).any()


def test_oracle_rejects_nonpositive_iterations():
    H = hstd_for("BCH_7_4_1_strip")
    with pytest.raises(ValueError):
        oracle.spa_decode(H, np.zeros((1, 7)), 0)
