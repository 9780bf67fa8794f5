"""BER/FER curve overlay against the reference's own Monte-Carlo run
(north_star: "BER curve overlaying the CPU reference at Eb/N0 1.0-3.0 dB";
SURVEY.md §8 f1).  The reference curve was measured by running
python_ldpc_app/main.py (tests/golden/gen_ber_curve.py); its RNG is
time-seeded, so parity is statistical: the reference's FER and BER at every
point must lie inside the central 99 % of the GPU's sampling distribution at
the reference's own frame count B (tests/ber_overlay.py)."""
import pytest

pytestmark = pytest.mark.gpu


def test_ber_curve_overlays_reference(gpu_available):
    import ber_overlay
    from conftest import hstd_for
    from ldpc_amd.device import Decoder, Graph

    dec = Decoder(Graph(hstd_for("wimax_576_0.5"), device=0), 65536)
    rows = ber_overlay.overlay(dec, groups=200)
    assert len(rows) == 5 and rows[0]["snr_db"] == 1.0 and rows[-1]["snr_db"] == 3.0
    for r in rows:
        print(r)
        assert r["fer_lo"] <= r["fer_ref"] <= r["fer_hi"], r
        assert r["ber_lo"] <= r["ber_ref"] <= r["ber_hi"], r
    # the curve falls: FER strictly decreasing over 1.0 -> 3.0 dB on the GPU
    fers = [r["fer_gpu"] for r in rows]
    assert all(a > b for a, b in zip(fers, fers[1:])), fers


def test_ber_curve_overlays_reference_north_star_code(gpu_available):
    """The same overlay on wimax_2304_0.5 (BASELINE config 3's code) at
    1.0 / 2.0 / 3.0 dB against the reference's own main.py run."""
    import ber_overlay
    from conftest import hstd_for
    from ldpc_amd.device import Decoder, Graph

    dec = Decoder(Graph(hstd_for("wimax_2304_0.5"), device=0), 12800)
    rows = ber_overlay.overlay(dec, groups=200, code="wimax_2304_0.5")
    assert [r["snr_db"] for r in rows] == [1.0, 2.0, 3.0]
    for r in rows:
        print(r)
        assert r["fer_lo"] <= r["fer_ref"] <= r["fer_hi"], r
        assert r["ber_lo"] <= r["ber_ref"] <= r["ber_hi"], r
    fers = [r["fer_gpu"] for r in rows]
    assert all(a > b for a, b in zip(fers, fers[1:])), fers


def test_ber_curve_overlays_reference_config4_code(gpu_available):
    """The same overlay on wimax_2304_0.75A (BASELINE config 4's code) at
    2.0 / 2.5 / 3.0 dB, where its FER moves (0.8 -> 0.07), against the
    reference's own main.py run (tests/golden/gen_ber_curve.py --code
    wimax_2304_0.75A: 48 / 64 / 96 frames).  Its failing frames at 3 dB carry
    few or no information-bit errors (the sign quirk of odd-degree rows,
    DESIGN.md §2), in the reference and on the GPU alike."""
    import ber_overlay
    from conftest import hstd_for
    from ldpc_amd.device import Decoder, Graph

    dec = Decoder(Graph(hstd_for("wimax_2304_0.75A"), device=0), 9600)
    rows = ber_overlay.overlay(dec, groups=200, code="wimax_2304_0.75A")
    assert [r["snr_db"] for r in rows] == [2.0, 2.5, 3.0]
    for r in rows:
        print(r)
        assert r["fer_lo"] <= r["fer_ref"] <= r["fer_hi"], r
        assert r["ber_lo"] <= r["ber_ref"] <= r["ber_hi"], r
    fers = [r["fer_gpu"] for r in rows]
    assert all(a > b for a, b in zip(fers, fers[1:])), fers
