"""Shared fixtures.  GPU tests are marked @pytest.mark.gpu and run on an MI355X;
everything else runs on the CPU (oracle vs golden vectors, host logic, ABI)."""
import glob
import os
import sys

import numpy as np
import pytest
from scipy import sparse

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "ldpc-simulator_amd")
ORACLE_DIR = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG_DIR, ORACLE_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)

# tolerance for fp64 LLRs / messages (BASELINE.json north_star: 1e-5 relative).
# atol covers values that cancel to ~0 where a relative bound is meaningless.
LLR_RTOL = 1e-5
LLR_ATOL = 1e-9

GOLDEN_SETS = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz")))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


def load_code_npz(name):
    return np.load(os.path.join(PKG_DIR, "ldpc_amd", "codes", f"{name}.npz"), allow_pickle=False)


_HSTD = {}


def hstd_for(name):
    """H_std for a committed code, built by the native builder (hash-checked in tests)."""
    if name not in _HSTD:
        import ldpc_amd
        c = load_code_npz(name)
        H = sparse.csr_matrix((c["h_data"], c["h_indices"], c["h_indptr"]), shape=(int(c["m"]), int(c["n"])))
        Hs, perm = ldpc_amd.build_standard_form(H)
        assert ldpc_amd.csr_fingerprint(Hs) == str(c["hstd_sha"])
        _HSTD[name] = Hs
    return _HSTD[name]


def load_golden(set_name):
    g = np.load(os.path.join(GOLDEN, f"{set_name}.npz"), allow_pickle=False)
    return {k: g[k] for k in g.files}


def assert_llr_close(actual, expected, what, slack=None):
    """|a-b| <= rtol*|b| + atol, or <= slack where the oracle measured that ONE
    ulp of tanh moves the value further (frames saturated at the +-CL clip,
    oracle.conditioning_slack); slack is ~0 for every natural-channel frame."""
    actual = np.asarray(actual, dtype=np.float64)
    expected = np.asarray(expected, dtype=np.float64)
    bad = ~np.isclose(actual, expected, rtol=LLR_RTOL, atol=LLR_ATOL)
    if slack is not None:
        bad &= ~(np.abs(actual - expected) <= np.asarray(slack))
    if bad.any():
        idx = np.argwhere(bad)[:5]
        raise AssertionError(f"{what}: {int(bad.sum())} values outside rtol={LLR_RTOL}: "
                             + ", ".join(f"{tuple(i)}: {actual[tuple(i)]!r} vs {expected[tuple(i)]!r}" for i in idx))


def max_rel(actual, expected):
    a, b = np.asarray(actual, np.float64), np.asarray(expected, np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300))) if a.size else 0.0


@pytest.fixture(scope="session")
def gpu_available():
    import ldpc_amd
    n = ldpc_amd.device_count()
    if n <= 0:
        pytest.fail("GPU test selected but no HIP device is visible (no CPU fallback exists)")
    return n
