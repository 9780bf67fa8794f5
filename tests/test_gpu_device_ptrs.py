"""LDPC_F_DEVICE_PTRS (include/ldpc_hip.h): every I/O buffer in device
memory, the decode asynchronous on the caller's stream.  Results must be
identical to the host-pointer path, chunked or not, tile-resident or split,
with and without the normalized-LLR outputs.

Device buffers and the stream come straight from the HIP runtime that
libldpc_hip.so runs on (hipMalloc / hipStreamCreate through ctypes), as a
C or cgo caller of the ABI would make them."""
import ctypes

import numpy as np
import pytest

from conftest import hstd_for
from test_gpu_parity import _random_llr

pytestmark = pytest.mark.gpu

H2D, D2H = 1, 2  # hipMemcpyHostToDevice, hipMemcpyDeviceToHost


class Hip:
    """The process's HIP runtime (the libamdhip64.so.7 libldpc_hip.so loaded)."""

    def __init__(self):
        from ldpc_amd import _lib
        _lib.lib()  # libldpc_hip.so first: its runtime is the one found below
        self.rt = ctypes.CDLL("libamdhip64.so.7")
        for f in ("hipMalloc", "hipFree", "hipMemcpy", "hipMemset", "hipStreamCreate", "hipStreamDestroy",
                  "hipStreamSynchronize", "hipDeviceSynchronize"):
            getattr(self.rt, f).restype = ctypes.c_int
        self.rt.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        self.rt.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
        self.rt.hipFree.argtypes = [ctypes.c_void_p]
        self.rt.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
        self.rt.hipStreamDestroy.argtypes = [ctypes.c_void_p]

    def ok(self, rc, what):
        assert rc == 0, f"{what}: hipError {rc}"


class DevBuf:
    """Device allocation with the shape/dtype of a numpy array."""

    def __init__(self, hip, shape, dtype, fill=None):
        self.hip, self.shape, self.dtype = hip, tuple(shape), np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape)) * self.dtype.itemsize
        self.p = ctypes.c_void_p()
        hip.ok(hip.rt.hipMalloc(ctypes.byref(self.p), ctypes.c_size_t(max(1, self.nbytes))), "hipMalloc")
        if fill is not None:
            self.upload(np.full(self.shape, fill, self.dtype))

    @classmethod
    def of(cls, hip, a):
        b = cls(hip, a.shape, a.dtype)
        b.upload(a)
        return b

    def data_ptr(self):
        return self.p.value

    def upload(self, a):
        a = np.ascontiguousarray(a, self.dtype)
        self.hip.ok(self.hip.rt.hipMemcpy(self.p, a.ctypes.data, self.nbytes, H2D), "hipMemcpy H2D")

    def numpy(self):
        out = np.empty(self.shape, self.dtype)
        self.hip.ok(self.hip.rt.hipMemcpy(out.ctypes.data, self.p, self.nbytes, D2H), "hipMemcpy D2H")
        return out

    def __del__(self):
        if self.p.value:
            self.hip.rt.hipFree(self.p)
            self.p = ctypes.c_void_p()


@pytest.fixture(scope="module")
def hip(gpu_available):
    return Hip()


def _decoder(code, frames):
    from ldpc_amd.device import Decoder, Graph
    return Decoder(Graph.cached(hstd_for(code)), frames)


@pytest.mark.parametrize("code,cap,B,T,snr,split", [
    ("wimax_576_0.5", 256, 200, 12, 1.5, False),   # tile-resident decoder, one chunk
    ("wimax_576_0.5", 128, 200, 12, 1.5, False),   # two chunks through 128 slots
    ("wimax_576_0.5", 128, 200, 8, 0.5, True),     # per-iteration CN/VN launches
    ("wimax_2304_0.75A", 64, 70, 5, 2.0, False),   # long rows (cn_kernel), ragged chunk
])
@pytest.mark.parametrize("with_nllr", [False, True])
def test_device_pointers_equal_host_path(hip, code, cap, B, T, snr, split, with_nllr):
    H = hstd_for(code)
    n = H.shape[1]
    llr = _random_llr(H, B, snr, seed=4242 + B + T)
    dec = _decoder(code, cap)
    ref = dec.decode(llr, T, nllr=with_nllr, post=True, hist=with_nllr, split=split)

    llr_d = DevBuf.of(hip, llr)
    z = DevBuf(hip, (B, n), np.uint8)
    conv = DevBuf(hip, (B,), np.int32)
    status = DevBuf(hip, (B,), np.int32)
    iters = DevBuf(hip, (B,), np.int32)
    post = DevBuf(hip, (B, n), np.float64)
    nl = DevBuf(hip, (B,), np.float64) if with_nllr else None
    hi = DevBuf(hip, (B, T), np.float64) if with_nllr else None
    s = ctypes.c_void_p()
    hip.ok(hip.rt.hipStreamCreate(ctypes.byref(s)), "hipStreamCreate")
    try:
        dec.decode_device(llr_d, T, z=z, conv=conv, status=status, post=post, nllr=nl, hist=hi, iters=iters,
                          split=split, stream=s.value)
        hip.ok(hip.rt.hipStreamSynchronize(s), "hipStreamSynchronize")
    finally:
        hip.rt.hipStreamDestroy(s)

    np.testing.assert_array_equal(z.numpy(), ref.z)
    np.testing.assert_array_equal(conv.numpy(), ref.conv)
    np.testing.assert_array_equal(status.numpy(), ref.status)
    np.testing.assert_array_equal(iters.numpy(), ref.iters)
    np.testing.assert_array_equal(post.numpy(), ref.post)
    if with_nllr:
        np.testing.assert_array_equal(nl.numpy(), ref.nllr)
        np.testing.assert_array_equal(hi.numpy(), ref.hist)


def test_device_pointers_some_outputs_null_stream(hip):
    """Only conv requested, null stream: the other outputs are not written."""
    code, B, T = "wimax_576_0.5", 96, 6
    llr = _random_llr(hstd_for(code), B, 2.0, seed=77)
    dec = _decoder(code, 128)
    ref = dec.decode(llr, T)
    conv = DevBuf(hip, (B,), np.int32, fill=-7)
    dec.decode_device(DevBuf.of(hip, llr), T, conv=conv)
    hip.ok(hip.rt.hipDeviceSynchronize(), "hipDeviceSynchronize")
    np.testing.assert_array_equal(conv.numpy(), ref.conv)


def test_device_pointers_reject_host_only_message_export(hip):
    from ldpc_amd import _lib
    from ldpc_amd._lib import LDPC_F_DEVICE_PTRS, LdpcError, check
    dec = _decoder("wimax_576_0.5", 64)
    llr = DevBuf(hip, (4, 576), np.float64, fill=0.0)
    msgs = np.empty((4, dec.graph.nnz))
    with pytest.raises(LdpcError, match="host-only"):
        check("ldpc_decode_f64", _lib.lib().ldpc_decode_f64(
            dec._h, 4, ctypes.c_void_p(llr.data_ptr()), 3, LDPC_F_DEVICE_PTRS, None, None, None, None, None, None,
            None, _lib.ptr(msgs), None))
