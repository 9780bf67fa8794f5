"""Parity at BASELINE.json's full sizes, through size-independent properties.

configs[1]  wimax_576_0.5, 65,536 frames, T=50:
   - counter identity: sum(iters) == sum(conv) + n_conv + (frames - n_conv) * T
   - additivity of the frame-index shards (what the multi-GPU run relies on)
   - a spot sample of frames from deep inside the batch == the oracle, bit-exact
   - every frame reported OK satisfies H_std (z^1) = 0 (round trip
     encode -> channel -> decode -> syndrome)
configs[2]  wimax_2304_0.5, T=50 + early termination, a 16,384-frame sub-batch
configs[3]  wimax_2304_0.75A sweep 1.0..4.0 dB
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


def _identity(c, T):
    frames, failed, err, sconv, nconv, _, iters = (int(x) for x in c)
    assert iters == sconv + nconv + (frames - nconv) * T
    assert failed == frames - nconv
    return frames, failed, err


@pytest.mark.parametrize("snr", [0.0, 2.0])
def test_576_full_batch_counters(gpu_available, snr):
    B, T = 65536, 50
    dec = _decoder("wimax_576_0.5", B)
    sig = oracle.sigma_for_snr(snr)
    whole = dec.mc_run(SEED, [sig], B, 0, T)[0]
    frames, failed, _ = _identity(whole, T)
    assert frames == B
    half_a = dec.mc_run(SEED, [sig], B // 2, 0, T)[0]
    half_b = dec.mc_run(SEED, [sig], B // 2, B // 2, T)[0]
    np.testing.assert_array_equal(whole, half_a + half_b)
    if snr == 0.0:
        assert failed / frames > 0.97  # reference FER 1.0 at 0 dB


def _syndrome_ok(H, z):
    return ((H @ (1 - z.astype(np.int64)).T) % 2).sum(axis=0) == 0


def test_576_full_batch_decode_vs_oracle_sample(gpu_available):
    code, B, T = "wimax_576_0.5", 65536, 50
    H = hstd_for(code)
    dec = _decoder(code, B)
    sig = oracle.sigma_for_snr(1.5)
    llr = np.empty((B, H.shape[1]))
    for s in range(0, B, 16384):  # the generator fills up to the decoder capacity
        _, llr[s:s + 16384] = dec.generate(SEED, 0, sig, s, 16384)
    r = dec.decode(llr, T)
    ok = r.status == 0
    assert _syndrome_ok(H, r.z[ok]).all()
    rng = np.random.default_rng(1)
    idx = np.sort(rng.choice(B, 48, replace=False))
    o = oracle.spa_decode(H, llr[idx], T)
    np.testing.assert_array_equal(r.z[idx], o["z"])
    np.testing.assert_array_equal(r.conv[idx], o["conv"])
    np.testing.assert_array_equal(r.status[idx], o["status"])


def test_2304_half_rate_subbatch(gpu_available):
    code, B, T = "wimax_2304_0.5", 16384, 50
    H = hstd_for(code)
    dec = _decoder(code, B)
    sig = oracle.sigma_for_snr(2.0)
    c = dec.mc_run(SEED, [sig], B, 0, T)[0]
    _identity(c, T)
    _, llr = dec.generate(SEED, 0, sig, 0, 64)
    r = dec.decode(llr, T)
    o = oracle.spa_decode(H, llr[:8], T)
    np.testing.assert_array_equal(r.z[:8], o["z"])
    np.testing.assert_array_equal(r.conv[:8], o["conv"])
    assert _syndrome_ok(H, r.z[r.status == 0]).all()


def test_2304_three_quarter_sweep(gpu_available):
    """FER is NOT monotone here, in the reference too: 83% of this code's H_std
    rows have odd degree, and the reference's check rule with its LLR sign
    convention sends wrong-sign saturated extrinsics, so from
    ~4 dB on no frame converges although the channel hard decisions are already
    error-free.  The GPU must reproduce that cliff exactly."""
    code, B, T = "wimax_2304_0.75A", 4096, 50
    H = hstd_for(code)
    k = H.shape[1] - H.shape[0]
    dec = _decoder(code, B)
    snrs = [1.0, 2.0, 3.0, 4.0]
    sig = [oracle.sigma_for_snr(s) for s in snrs]
    ctr = dec.mc_run(SEED, sig, B, 0, T)
    for c in ctr:
        _identity(c, T)
    # the first 24 frames of the 3 dB and 4 dB points == the oracle, counter for counter
    small = dec.mc_run(SEED, sig, 24, 0, T)
    for p in (2, 3):
        u, llr = dec.generate(SEED, p, sig[p], 0, 24)
        o = oracle.spa_decode(H, llr, T)
        want = oracle.main_counters(u, o["z"], o["status"], o["conv"], iters=o["iters"])
        np.testing.assert_array_equal(small[p][[0, 1, 2, 3, 4, 6]], want[[0, 1, 2, 3, 4, 6]])
    assert ctr[2][1] / B < 0.15 and ctr[3][1] / B > 0.95  # mostly converges at 3 dB, never at 4 dB
    del k
