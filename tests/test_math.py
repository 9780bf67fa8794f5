"""The fp64 math of the check-node update, checked on the CPU.

np_tanh   (csrc/spa_math.h, the code the GPU runs, host build) and the
          oracle's restatement must equal the reference's np.tanh bit for bit.
atanh_f   must be faithful (<= 1 ulp) everywhere on [0, CL] and agree with
          numpy's arctanh (what the reference calls) on > 99% of inputs.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

CL = 0.99999999999999878
BUILD = os.path.join(ROOT, "tests", "_build")


@pytest.fixture(scope="module")
def host_math():
    os.makedirs(BUILD, exist_ok=True)
    so = os.path.join(BUILD, "libspa_math_host.so")
    src = os.path.join(ROOT, "tests", "native", "math_host.cpp")
    hdr = os.path.join(ROOT, "ldpc-simulator_amd", "csrc", "spa_math.h")
    tabs = os.path.join(ROOT, "ldpc-simulator_amd", "csrc", "spa_math_tables.h")
    if not os.path.exists(so) or os.path.getmtime(so) < max(map(os.path.getmtime, (src, hdr, tabs))):
        subprocess.run(["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-arch=gfx950", "-O2", "-std=c++17",
                        "-ffp-contract=off", "-fPIC", "-shared", "-o", so, src], check=True)
    L = ctypes.CDLL(so)
    for fn in (L.host_np_tanh, L.host_atanh):
        fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long]
    return L


def _run(fn, x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty_like(x)
    fn(x.ctypes.data, y.ctypes.data, len(x))
    return y


def _tanh_inputs(n=1_500_000, seed=3):
    rng = np.random.default_rng(seed)
    return np.concatenate([rng.uniform(-17.5, 17.5, n // 2), rng.uniform(-1, 1, n // 4),
                           rng.uniform(-1e-3, 1e-3, n // 8), rng.uniform(-40, 40, n // 8),
                           [0.0, -0.0, 0.1875, 0.25, 24.0, -24.0, 17.5, -17.5, 1e-300]])


def test_device_tanh_equals_numpy_tanh(host_math):
    x = _tanh_inputs()
    y = _run(host_math.host_np_tanh, x)
    np.testing.assert_array_equal(y, np.tanh(x))
    assert np.signbit(_run(host_math.host_np_tanh, np.array([-0.0]))[0])


def test_tanh_output_clip_equals_input_clip(host_math):
    """cn_common.h cn_tanh: clip(np_tanh(d), -CL, CL) is the reference's
    input clip (spa_decoder.py:138-146: d > 17.5 -> CL, d < -17.5 -> -CL)
    bit for bit -- np.tanh(17.5) == CL and np_tanh is monotone across +-17.5."""
    assert np.tanh(17.5) == CL and _run(host_math.host_np_tanh, np.array([17.5]))[0] == CL
    base = np.float64(17.5).view(np.int64)
    k = np.arange(2_000_000, dtype=np.int64)
    rng = np.random.default_rng(11)
    x = np.concatenate([(base + k).view(np.float64), (base - k).view(np.float64)])
    x = np.concatenate([x, -x, rng.uniform(-40, 40, 1_000_000),
                        10 ** rng.uniform(0, 308, 200_000) * rng.choice([-1, 1], 200_000),
                        [np.inf, -np.inf, 1.7e308, -1.7e308, 24.0, -24.0]])
    y = _run(host_math.host_np_tanh, x)
    sel = np.where(x > 17.5, CL, np.where(x < -17.5, -CL, y))
    np.testing.assert_array_equal(np.clip(y, -CL, CL).view(np.int64), sel.view(np.int64))


def test_tanh_half_clipped_equals_reference_clip(host_math):
    """spa_math.h tanh_half_clipped(M) (what the kernels run) == the
    reference's d = M/2; d > 17.5 -> CL, d < -17.5 -> -CL, else np.tanh(d)
    (spa_decoder.py:138-146), bit for bit, including -0.0 and the 2e6
    consecutive doubles each side of +-17.5 (= M of +-35)."""
    fn = host_math.host_tanh_half_clipped
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long]
    base = np.float64(35.0).view(np.int64)
    k = np.arange(2_000_000, dtype=np.int64)
    rng = np.random.default_rng(12)
    m = np.concatenate([(base + k).view(np.float64), (base - k).view(np.float64)])
    m = np.concatenate([m, -m, rng.uniform(-80, 80, 1_000_000), rng.uniform(-2, 2, 500_000),
                        10 ** rng.uniform(-300, 308, 200_000) * rng.choice([-1, 1], 200_000),
                        [0.0, -0.0, 35.0, -35.0, 48.0, -48.0, 1e-320, 1.7e308, -1.7e308]])
    d = m / 2.0
    want = np.where(d > 17.5, CL, np.where(d < -17.5, -CL, np.tanh(d)))
    got = _run(fn, m)
    np.testing.assert_array_equal(got.view(np.int64), want.view(np.int64))


def test_oracle_tanh_equals_numpy_tanh():
    import oracle
    x = _tanh_inputs(400_000, seed=9)
    np.testing.assert_array_equal(oracle.np_tanh(x), np.tanh(x))


def _atanh_inputs(n=1_000_000, seed=4):
    rng = np.random.default_rng(seed)
    q = np.concatenate([rng.uniform(-1, 1, n // 2), 1 - 10 ** rng.uniform(-15.9, -0.3, n // 4),
                        rng.uniform(-0.05, 0.05, n // 8), 10 ** rng.uniform(-300, -1, n // 8),
                        [0.0, 2.0 ** -5, -(2.0 ** -5), 0.5, -0.5, CL, -CL]])
    return np.clip(q, -CL, CL)


def test_device_atanh_is_faithful_and_matches_numpy(host_math):
    q = _atanh_inputs()
    y = _run(host_math.host_atanh, q)
    libm = ctypes.CDLL("libm.so.6")
    libm.atanhl.restype = ctypes.c_longdouble
    libm.atanhl.argtypes = [ctypes.c_longdouble]
    sub = q[:: 25]
    exact = np.array([float(libm.atanhl(float(v))) for v in sub])  # correctly rounded w.h.p.
    ulps = np.abs(y[:: 25] - exact) / np.spacing(np.abs(exact))
    assert ulps.max() <= 1.0, ulps.max()
    assert np.mean(y[:: 25] == exact) > 0.999
    assert np.mean(y == np.arctanh(q)) > 0.98  # numpy (SVML) is itself ~97% CR below 0.1
    np.testing.assert_array_equal(np.signbit(y), np.signbit(q))


def test_atanh_is_identity_below_2_pow_minus_27(host_math):
    """spa_math.h kAtanhIdent: atanh_f(q) == q bit for bit for |q| < 2^-27 (the
    kernels' E_new = 2q fast path for a wavefront whose quotients are all that
    small), over the 2e6 doubles below 2^-27, log-uniform values down to the
    subnormals, and +-0.0; and not much beyond it ([2^-26, 2^-25) already
    holds values where it differs)."""
    top = np.float64(2.0 ** -27).view(np.int64)
    k = np.arange(1, 2_000_001, dtype=np.int64)
    rng = np.random.default_rng(13)
    q = np.concatenate([(top - k).view(np.float64), 2.0 ** rng.uniform(-1074, -27, 1_000_000),
                        [0.0, 5e-324, 2.2250738585072014e-308]])
    q = np.concatenate([q, -q])
    y = _run(host_math.host_atanh, q)
    np.testing.assert_array_equal(y.view(np.int64), q.view(np.int64))
    w = rng.uniform(2.0 ** -26, 2.0 ** -25, 100_000)
    assert (_run(host_math.host_atanh, w) != w).any()


def test_atanh_is_odd_for_the_saturation_memo(host_math):
    """tile8.hip t8_p3 (LDPC_T8_SATMEMO) gives a slot whose every lane has
    |q| == |q of slot 0| slot 0's E_new with the slot's own sign.  That is
    exact iff E(q) = 2 atanh_f(clip_cl(q)) is odd bit for bit (clip_cl is
    fmin/fmax: symmetric) -- and, where slot 0 took the 2q branch (every
    |q| < 2^-27), iff atanh_f(q) == q there (asserted last)."""
    rng = np.random.default_rng(11)
    q = np.concatenate([rng.uniform(0, CL, 400_000), 10.0 ** rng.uniform(-300, 0, 200_000),
                        CL - rng.uniform(0, 1e-12, 1000), [CL, 0.0, 2.0 ** -27, 2.0 ** -5, 0.5]])
    q = np.minimum(q, CL)
    pos = _run(host_math.host_atanh, q)
    neg = _run(host_math.host_atanh, -q)
    assert np.array_equal(neg.view(np.uint64), (-pos).view(np.uint64))
    small = q[q < 2.0 ** -27]
    assert np.array_equal(_run(host_math.host_atanh, small), small)
