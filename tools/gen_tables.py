#!/usr/bin/env python3
"""Generate the constant tables of the decoder's fp64 math (spa_math_tables.h).

1. numpy's float64 tanh.  The reference computes `np.tanh(d)` (spa_decoder.py:145)
   with numpy 2.2.6, whose float64 tanh (SIMD dispatch AVX512_SKX,
   numpy/_core/src/umath/loops_hyperbolic.dispatch) is: 16 intervals selected by
   the exponent and top mantissa bit of |x|, y = |x| - b[i], and a degree-16
   polynomial in y evaluated by Horner with fused multiply-adds, c16 down to
   c0; |x| >= 24 (and huge/inf) -> 1.0; the sign of x is OR-ed back in.  The
   per-interval constants (b, c0..c16) are numpy's published coefficient
   table; they are read here from the installed numpy build and the
   restatement is checked against np.tanh bit for bit before anything is
   written (tests/test_math.py re-checks on every CPU run).

2. A 128-entry natural-log table (invc, -log(invc) as a double-double) for the
   decoder's log-based atanh (spa_math.h atanh_f), computed with `decimal`.

Usage: python tools/gen_tables.py   (rewrites the two headers below)
"""
import ctypes
import os
import struct
import subprocess
import sys
import tempfile
from decimal import Decimal, getcontext

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT_PRODUCT = os.path.join(ROOT, "ldpc-simulator_amd", "csrc", "spa_math_tables.h")
OUT_ORACLE = os.path.join(ROOT, "oracle", "numpy_tanh_table.h")
NUMPY_SO = os.path.join(os.path.dirname(np.__file__), "_core",
                        "_multiarray_umath.cpython-310-x86_64-linux-gnu.so")


def find_numpy_tanh_table():
    """Locate numpy's [18][16] float64 tanh table: row 0 = b, rows 1.. = c0..c16.

    Anchors: b row = {0, 0.21875, 0.3125, ..., 20, 0}; the c3 row starts with -1/3.
    (numpy keeps a double-double c0 split; only the high part is used by the
    float64 kernel, which the bit-exact check below confirms.)
    """
    data = open(NUMPY_SO, "rb").read()
    b_row = struct.pack("<16d", 0.0, 0.21875, 0.3125, 0.4375, 0.625, 0.875, 1.25, 1.75, 2.5, 3.5,
                        5.0, 7.0, 10.0, 14.0, 20.0, 0.0)
    off = data.find(b_row)
    if off < 0:
        raise SystemExit("numpy tanh breakpoint row not found in " + NUMPY_SO)
    rows = [struct.unpack("<16Q", data[off + 128 * r: off + 128 * (r + 1)]) for r in range(19)]
    # rows: 0 b, 1 c0(hi), 2 c0(lo, unused by the f64 kernel), 3.. c1..c16
    b, c0, _c0lo = rows[0], rows[1], rows[2]
    cs = [c0] + rows[3:19]
    assert struct.unpack("<d", struct.pack("<Q", cs[3][0]))[0] == -1.0 / 3.0
    return b, cs  # cs[p] = coefficient of y^p, p = 0..16


C_CHECK = r"""
#include <math.h>
#include <stdint.h>
#include <string.h>
extern const unsigned long long B[16], C[17][16];
static double d(unsigned long long u) { double x; memcpy(&x, &u, 8); return x; }
double t(double x) {
    uint64_t ux; memcpy(&ux, &x, 8);
    uint64_t nd = ux & 0x7ff8000000000000ULL;
    int32_t hi = (int32_t)(nd >> 32) - 0x3fc00000;
    hi = hi < 0 ? 0 : (hi > 0x780000 ? 0x780000 : hi);
    int i = (uint32_t)hi >> 19;
    double y = fabs(x) - d(B[i]);
    double r = fma(d(C[16][i]), y, d(C[15][i]));
    for (int p = 14; p >= 0; --p) r = fma(r, y, d(C[p][i]));
    if (nd > 0x7fe0000000000000ULL) r = 1.0;
    uint64_t ur; memcpy(&ur, &r, 8); ur |= ux & 0x8000000000000000ULL; memcpy(&r, &ur, 8);
    return r;
}
void run(const double *x, double *y, long n) { for (long k = 0; k < n; ++k) y[k] = t(x[k]); }
"""


def verify(b, cs, n=3_000_000):
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "c.c")
        with open(src, "w") as fh:
            fh.write(C_CHECK)
            fh.write("const unsigned long long B[16] = {%s};\n" % ",".join("0x%016xULL" % v for v in b))
            fh.write("const unsigned long long C[17][16] = {%s};\n" % ",".join(
                "{" + ",".join("0x%016xULL" % v for v in row) + "}" for row in cs))
        so = os.path.join(td, "c.so")
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-shared", "-fPIC", "-o", so, src, "-lm"], check=True)
        L = ctypes.CDLL(so)
        L.run.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long]
        rng = np.random.default_rng(1)
        x = np.concatenate([rng.uniform(-1, 1, n // 3), rng.uniform(-30, 30, n // 3),
                            rng.uniform(-17.5, 17.5, n // 3), [0.0, -0.0, 24.0, 1e300, np.inf]])
        y = np.empty_like(x)
        L.run(x.ctypes.data, y.ctypes.data, len(x))
        bad = int((y != np.tanh(x)).sum())
        if bad:
            raise SystemExit(f"restated numpy tanh differs from np.tanh on {bad} inputs")
        return len(x)


def log_table(nbits=7):
    """glibc-style log reduction: x = 2^k z, z in [OFF, 2*OFF), i = top bits of z-OFF."""
    getcontext().prec = 80
    N = 1 << nbits
    OFF = 0x3FE6000000000000
    rows = []
    for i in range(N):
        lo = OFF + (i << (52 - nbits))
        hi = OFF + ((i + 1) << (52 - nbits))
        zlo = struct.unpack("<d", struct.pack("<Q", lo))[0]
        zhi = struct.unpack("<d", struct.pack("<Q", hi))[0]  # i = N-1: OFF + 2^52 = 2*OFF
        c = (Decimal(zlo) + Decimal(zhi)) / 2
        invc = float(1 / c)
        if zlo <= 1.0 < zhi:  # the interval holding 1.0: invc = 1 exactly -> log(z) = log1p(z-1)
            invc = 1.0
        L = -(Decimal(invc).ln())
        # hi on a 2^-43 grid so that k*Ln2hi + hi is exact in double (|.| < 2^10);
        # lo carries the rest (double-double)
        hi_ = float((L * (2 ** 43)).to_integral_value() / (2 ** 43))
        lo_ = float(L - Decimal(hi_))
        rows.append((invc, hi_, lo_))
    return rows


def main():
    b, cs = find_numpy_tanh_table()
    n = verify(b, cs)
    print(f"numpy tanh restatement verified bit-exact on {n} inputs")
    logt = log_table()

    def hx(u):
        return "0x%016xULL" % u

    def dbits(x):
        return struct.unpack("<Q", struct.pack("<d", x))[0]

    hdr = [
        "// GENERATED by tools/gen_tables.py -- do not edit.",
        "// (1) numpy 2.2.6 float64 tanh coefficient table (loops_hyperbolic, AVX512_SKX",
        "//     dispatch): kTanhB[i] = interval base b, kTanhC[p][i] = coefficient of y^p,",
        "//     y = |x| - b.  Restated algorithm verified bit-exact against np.tanh.",
        "// (2) log table for the decoder's log-based atanh: 128 x {invc, -log(invc) hi, lo}.",
        "#pragma once",
        "#include <cstdint>",
        "namespace ldpc {",
        "namespace tab {",
        "constexpr uint64_t kTanhB[16] = {%s};" % ", ".join(hx(v) for v in b),
        "constexpr uint64_t kTanhC[17][16] = {",
    ]
    for p, row in enumerate(cs):
        hdr.append("    {%s},  // c%d" % (", ".join(hx(v) for v in row), p))
    hdr.append("};")
    hdr.append("constexpr uint64_t kLog[128][3] = {  // invc, logc_hi, logc_lo")
    for invc, h, lo in logt:
        hdr.append("    {%s, %s, %s}," % (hx(dbits(invc)), hx(dbits(h)), hx(dbits(lo))))
    hdr.append("};")
    hdr.append("}  // namespace tab")
    hdr.append("}  // namespace ldpc")
    with open(OUT_PRODUCT, "w") as fh:
        fh.write("\n".join(hdr) + "\n")

    ohdr = [
        "/* GENERATED by tools/gen_tables.py -- numpy 2.2.6 float64 tanh table (see",
        " * spa_oracle.c: the reference's np.tanh, restated).  B[i] = interval base,",
        " * C[p][i] = coefficient of y^p. */",
        "static const unsigned long long NP_TANH_B[16] = {%s};" % ", ".join(hx(v) for v in b),
        "static const unsigned long long NP_TANH_C[17][16] = {",
    ]
    for row in cs:
        ohdr.append("    {%s}," % ", ".join(hx(v) for v in row))
    ohdr.append("};")
    with open(OUT_ORACLE, "w") as fh:
        fh.write("\n".join(ohdr) + "\n")
    print("wrote", OUT_PRODUCT, "and", OUT_ORACLE)


if __name__ == "__main__":
    sys.exit(main())
