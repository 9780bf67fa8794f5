"""The C-ABI library loads and exports every symbol include/ldpc_hip.h declares.

No compute calls here: without a GPU the decode entry points must FAIL (there
is no CPU fallback), which is also checked.
"""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import ldpc_amd
from ldpc_amd import _lib
from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "ldpc_hip.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ldpc_[a-z0-9_]+)\s*\(", txt)))


def test_header_and_binding_agree():
    assert declared_symbols() == sorted(_lib.EXPORTED)


def test_library_exports_every_declared_symbol():
    L = ctypes.CDLL(_lib.LIB_PATH)
    for sym in declared_symbols():
        assert hasattr(L, sym), sym
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    for sym in declared_symbols():
        assert re.search(rf"\bT {sym}\b", out), f"{sym} not exported with C linkage"


def test_library_has_gfx950_code_object():
    # the shared object carries its device code in the .hip_fatbin bundle
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"__CLANG_OFFLOAD_BUNDLE__" in data
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_abi_version():
    assert _lib.lib().ldpc_abi_version() == 5


def test_no_gpu_means_loud_failure():
    if ldpc_amd.device_count() > 0:
        pytest.skip("GPU present: covered by the gpu tests")
    H = np.array([0, 2], dtype=np.int32), np.array([0, 1], dtype=np.int32)
    h = ctypes.c_void_p()
    rc = _lib.lib().ldpc_graph_create(1, 2, _lib.i32p(H[0]), _lib.i32p(H[1]), -1, ctypes.byref(h))
    assert rc == -5  # LDPC_EDEVICE
    assert b"no HIP device" in _lib.lib().ldpc_last_error()


def test_graph_create_rejects_unsorted_rows():
    """Checked before any device call: the product order must be ascending."""
    rp = np.array([0, 2], dtype=np.int32)
    ci = np.array([1, 0], dtype=np.int32)
    h = ctypes.c_void_p()
    rc = _lib.lib().ldpc_graph_create(1, 2, _lib.i32p(rp), _lib.i32p(ci), -1, ctypes.byref(h))
    assert rc == -22


def test_decode_rejects_bad_args_without_touching_gpu():
    L = _lib.lib()
    assert L.ldpc_decode_f64(None, 1, None, 5, 0, None, None, None, None, None, None, None, None, None) == -22
