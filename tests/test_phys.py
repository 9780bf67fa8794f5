"""Physical mode: standard SPA on the sparse graph H[:, perm]
with the sign convention fixed, fp32, LDS-resident.  OUR design -- no
reference parity by construction; checked against its CPU restatement
(oracle/phys_oracle.c) and for decoding behaviour."""
import numpy as np
import pytest

import ldpc_amd
import oracle
from ldpc_amd import montecarlo as mc

SEED = 20260213


def _code(name):
    edd = ldpc_amd.load_committed_code(name)
    return edd, edd.physical_matrix()


@pytest.mark.parametrize("name", ["wimax_576_0.5", "wimax_2304_0.5", "wimax_2304_0.75A"])
def test_physical_graph_is_the_same_code(name):
    edd, Hp = _code(name)
    u = np.random.default_rng(0).integers(0, 2, size=(6, edd._k))
    c = edd.encode(u)
    assert not ((Hp @ c.T.astype(np.int64)) % 2).any()
    assert Hp.nnz < edd._h_std.nnz / 20  # sparse ALIST graph, not the RREF


def test_oracle_physical_decodes_clean_and_noisy_frames():
    edd, Hp = _code("wimax_576_0.5")
    u, c, llr = oracle.generate_frames(edd._h_std, SEED, 0, mc.sigma_for_snr(0.0), 0, 64)
    r = oracle.phys_decode(Hp, llr, 50)
    assert (r["status"] == 0).all()
    np.testing.assert_array_equal(r["z"] ^ 1, c)  # z = bit estimate ^ 1 (reference convention)
    # waterfall near -2.5 dB on the reference axis (noise std sigma^2): FER
    # ~1 at -4 dB, ~0 at -1.5 dB, in between at -2.5 dB
    fers = []
    for snr in (-4.0, -2.5, -1.5):
        _, _, llr = oracle.generate_frames(edd._h_std, SEED, 1, mc.sigma_for_snr(snr), 0, 96)
        fers.append(np.mean(oracle.phys_decode(Hp, llr, 50)["status"] != 0))
    assert fers[0] > 0.9 and 0.05 < fers[1] < 0.95 and fers[2] < 0.05, fers


@pytest.mark.gpu
@pytest.mark.parametrize("name,snr", [("wimax_576_0.5", -6.0), ("wimax_2304_0.5", -6.5), ("wimax_2304_0.75A", -3.0)])
def test_gpu_physical_matches_restatement(gpu_available, name, snr):
    from ldpc_amd.device import Graph, phys_decode
    edd, Hp = _code(name)
    _, c, llr = oracle.generate_frames(edd._h_std, SEED, 2, mc.sigma_for_snr(snr), 0, 96)
    g = phys_decode(Graph.cached(Hp), llr, 50, post=True)
    o = oracle.phys_decode(Hp, llr, 50)
    # ulp-level expm1f/log1pf differences may flip a marginal frame, never many
    same = (g.z == o["z"]).all(axis=1) & (g.conv == o["conv"])
    assert same.mean() >= 0.95, same.mean()
    agree = same.nonzero()[0]
    np.testing.assert_allclose(g.post[agree], o["post"][agree], rtol=2e-3, atol=2e-3)


@pytest.mark.gpu
def test_gpu_physical_mc_counters(gpu_available):
    from ldpc_amd.device import Decoder, Graph
    edd, Hp = _code("wimax_576_0.5")
    dec = Decoder(Graph.cached(edd._h_std), 2048)
    gp = Graph.cached(Hp)
    sig = [mc.sigma_for_snr(s) for s in (-7.0, -5.0, 0.0)]
    ctr = dec.phys_mc_run(gp, SEED, sig, 2048, 0, 50)
    for c in ctr:
        frames, failed, err, sconv, nconv, _, iters = (int(x) for x in c)
        assert frames == 2048 and failed == frames - nconv
        assert iters == sconv + nconv + failed * 50
    fers = ctr[:, 1] / ctr[:, 0]
    assert fers[0] >= fers[1] >= fers[2] == 0.0  # physical mode: FER falls with SNR
    # counters == restatement on the same device-generated frames
    u, llr = dec.generate(SEED, 1, sig[1], 0, 256)
    o = oracle.phys_decode(Hp, llr, 50)
    small = dec.phys_mc_run(gp, SEED, sig, 256, 0, 50)[1]
    want = oracle.main_counters(u, o["z"], o["status"], o["conv"], iters=o["iters"])
    assert abs(int(small[1]) - int(want[1])) <= 3  # failed frames (marginal-frame flips only)
