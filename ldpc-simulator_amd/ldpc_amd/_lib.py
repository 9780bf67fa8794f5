"""ctypes binding of libldpc_hip.so (C ABI: include/ldpc_hip.h).

The shared library is built in-tree (``ldpc-simulator_amd/csrc/Makefile`` ->
``ldpc_amd/libldpc_hip.so``).  There is no fallback: if the library is
missing, or a compute entry point is called without a GPU, this module raises.

Fork safety (main.py:221 builds an SPA_Decoder in the parent, then
main.py:248-256 forks a ProcessPoolExecutor whose workers build their own,
main.py:78; adaptive.py:227-282 likewise).  Loading the library does not start
the HIP runtime; the first call through ``gpu()`` does, and records the pid.
A process forked from a parent that had started HIP cannot use the inherited
runtime, so ``gpu()`` in such a child raises LdpcError instead of touching
it; a child of a parent that never did (the main.py pattern: construction is
HIP-free, see spa_decoder.py) starts its own.
"""
import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LDPC_HIP_LIB", os.path.join(_HERE, "libldpc_hip.so"))

LDPC_F_NLLR = 0x1
LDPC_F_DEVICE_PTRS = 0x2
LDPC_F_STATIC = 0x4
LDPC_F_PHYS_HBM = 0x8
LDPC_F_SPLIT = 0x10
LDPC_F_TEST_ZERO = 0x20  # test only: frame-source erasures (include/ldpc_hip.h)
LDPC_MC_NCOUNT = 7
LDPC_EINVAL = -22  # include/ldpc_hip.h error codes used on the Python side
LDPC_ERANGE = -34

# every symbol include/ldpc_hip.h declares
EXPORTED = (
    "ldpc_last_error", "ldpc_abi_version", "ldpc_device_count",
    "ldpc_hstd_build", "ldpc_hstd_get", "ldpc_hstd_free",
    "ldpc_graph_create", "ldpc_graph_destroy", "ldpc_graph_info", "ldpc_cn_kernel_name",
    "ldpc_phys_kernel_name", "ldpc_tile_lds_bytes", "ldpc_tile_kernel_name",
    "ldpc_decoder_bytes", "ldpc_decoder_create", "ldpc_decoder_destroy", "ldpc_decoder_capacity",
    "ldpc_decode_f64", "ldpc_generate_frames", "ldpc_mc_run", "ldpc_frame_order",
    "ldpc_profile_enable", "ldpc_profile_read", "ldpc_rare_rows_read",
    "ldpc_phys_lds_bytes", "ldpc_phys_decode", "ldpc_phys_mc_run",
    "ldpc_comm_unique_id", "ldpc_comm_init", "ldpc_comm_allreduce", "ldpc_comm_barrier", "ldpc_comm_destroy",
    "ldpc_device_synchronize",
)


class LdpcError(RuntimeError):
    """A libldpc_hip.so call failed (the message is ldpc_last_error())."""

    def __init__(self, fn, code, msg):
        super().__init__(f"{fn} failed ({code}): {msg}")
        self.code = code


_lock = threading.Lock()
_lib = None
_gpu_pid = None  # pid of the process that started the HIP runtime through gpu()
LDPC_EFORK = -100  # Python-side code: HIP was started in a parent process before fork

P = ctypes.POINTER
c_i32, c_i64, c_u32, c_u64, c_dbl, c_vp = (ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32,
                                           ctypes.c_uint64, ctypes.c_double, ctypes.c_void_p)


def _declare(lib):
    sig = {
        "ldpc_last_error": (ctypes.c_char_p, []),
        "ldpc_abi_version": (ctypes.c_int, []),
        "ldpc_device_count": (ctypes.c_int, []),
        "ldpc_hstd_build": (ctypes.c_int, [c_i32, c_i32, P(c_i32), P(c_i32), P(c_vp)]),
        "ldpc_hstd_get": (ctypes.c_int, [c_vp, P(c_i32), P(c_i32), P(c_i64), P(P(c_i32)),
                                         P(P(c_i32)), P(P(c_i32))]),
        "ldpc_hstd_free": (None, [c_vp]),
        "ldpc_graph_create": (ctypes.c_int, [c_i32, c_i32, P(c_i32), P(c_i32), c_i32, P(c_vp)]),
        "ldpc_graph_destroy": (ctypes.c_int, [c_vp]),
        "ldpc_graph_info": (ctypes.c_int, [c_vp, P(c_i32), P(c_i32), P(c_i64), P(c_i32), P(c_i32)]),
        "ldpc_cn_kernel_name": (ctypes.c_char_p, [c_vp]),
        "ldpc_phys_kernel_name": (ctypes.c_char_p, [c_vp, ctypes.c_uint32]),
        "ldpc_tile_lds_bytes": (ctypes.c_int64, [c_vp]),
        "ldpc_tile_kernel_name": (ctypes.c_char_p, [c_vp]),
        "ldpc_decoder_bytes": (c_i64, [c_vp, c_i32]),
        "ldpc_decoder_create": (ctypes.c_int, [c_vp, c_i32, P(c_vp)]),
        "ldpc_decoder_destroy": (ctypes.c_int, [c_vp]),
        "ldpc_decoder_capacity": (c_i32, [c_vp]),
        "ldpc_decode_f64": (ctypes.c_int, [c_vp, c_i32, c_vp, c_i32, c_u32, c_vp, c_vp, c_vp, c_vp,
                                           c_vp, c_vp, c_vp, c_vp, c_vp]),
        "ldpc_generate_frames": (ctypes.c_int, [c_vp, c_u64, c_i32, c_dbl, c_i64, c_i32, c_u32,
                                                c_vp, c_vp, c_vp]),
        "ldpc_mc_run": (ctypes.c_int, [c_vp, c_u64, c_i32, P(c_dbl), c_i64, c_i64, c_i32, c_u32,
                                       P(c_i64), c_vp]),
        "ldpc_frame_order": (ctypes.c_int, [c_vp, c_u64, c_i32, c_dbl, c_i64, c_i32, c_vp, c_vp]),
        "ldpc_profile_enable": (ctypes.c_int, [c_vp, ctypes.c_int]),
        "ldpc_phys_lds_bytes": (c_i64, [c_vp]),
        "ldpc_phys_decode": (ctypes.c_int, [c_vp, c_i32, c_vp, c_i32, c_u32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
        "ldpc_phys_mc_run": (ctypes.c_int, [c_vp, c_vp, c_u64, c_i32, P(c_dbl), c_i64, c_i64, c_i32, c_u32,
                                            P(c_i64), c_vp]),
        "ldpc_profile_read": (ctypes.c_int, [c_vp, P(c_dbl), P(c_i64)]),
        "ldpc_rare_rows_read": (ctypes.c_int, [c_vp, P(c_i64)]),
        "ldpc_comm_unique_id": (ctypes.c_int, [c_vp]),
        "ldpc_comm_init": (ctypes.c_int, [c_vp, c_i32, c_i32, c_i32, P(c_vp)]),
        "ldpc_comm_allreduce": (ctypes.c_int, [c_vp, c_vp, c_i64, c_i32, c_i32, c_u32, c_vp]),
        "ldpc_comm_barrier": (ctypes.c_int, [c_vp]),
        "ldpc_comm_destroy": (ctypes.c_int, [c_vp]),
        "ldpc_device_synchronize": (ctypes.c_int, [c_i32]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def lib():
    """Load (once) and return the ctypes handle; raises if the .so is absent."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"libldpc_hip.so not found at {LIB_PATH}: build it with "
                    "`make -C ldpc-simulator_amd/csrc` (or __graft_entry__.build()). "
                    "There is no CPU fallback.")
            handle = ctypes.CDLL(LIB_PATH)
            _declare(handle)
            _lib = handle
    return _lib


def gpu():
    """The library handle for calls that use the HIP runtime (every entry point
    except ldpc_hstd_*, ldpc_last_error, ldpc_abi_version).  Raises in a
    process forked after its parent started HIP (see the module docstring)."""
    global _gpu_pid
    pid = os.getpid()
    if _gpu_pid is not None and _gpu_pid != pid:
        raise LdpcError("gpu", LDPC_EFORK,
                        f"the HIP runtime was started in process {_gpu_pid} before it forked this process "
                        f"({pid}); a forked child cannot use it.  Construct SPA_Decoder objects freely in the "
                        "parent (construction does not start HIP) but decode only in the workers, or use the "
                        "'spawn' start method")
    h = lib()
    _gpu_pid = pid
    return h


def hip_started_here():
    """Whether this process has started the HIP runtime through gpu()."""
    return _gpu_pid == os.getpid()


def check(fn_name, rc):
    if rc != 0:
        msg = lib().ldpc_last_error()  # thread-local string, no HIP
        raise LdpcError(fn_name, rc, msg.decode() if msg else "")
    return rc


def ptr(a):
    """Address of a C-contiguous numpy array (or None -> NULL)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
    return a.ctypes.data


def i32p(a):
    return a.ctypes.data_as(P(c_i32))


def device_count():
    return int(gpu().ldpc_device_count())


def as_i32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.int32))
