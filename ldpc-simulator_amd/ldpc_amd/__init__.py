"""ldpc_amd -- MI355X-native SPA (belief-propagation) LDPC decoder.

Host side of the drop-in for python_ldpc_app/spa_decoder.py; the compute is
the HIP library libldpc_hip.so (ldpc-simulator_amd/csrc), bound with ctypes.
Import this package with ``ldpc-simulator_amd`` on sys.path (the directory name
is not a valid Python identifier; the reference itself runs as flat modules on
sys.path, python_ldpc_app/main.py).
"""
from ._lib import LdpcError, device_count, lib  # noqa: F401
from .code import EncoderDecoderData, build_standard_form, csr_fingerprint, load_committed_code  # noqa: F401
from .enums import Result  # noqa: F401
from .settings import Settings  # noqa: F401

__all__ = ["EncoderDecoderData", "Settings", "Result", "SPA_Decoder", "Graph", "Decoder",
           "build_standard_form", "csr_fingerprint", "load_committed_code", "device_count", "LdpcError"]


def __getattr__(name):  # lazy: the decoder classes touch the GPU only when used
    if name == "SPA_Decoder":
        from .spa_decoder import SPA_Decoder
        return SPA_Decoder
    if name in ("Graph", "Decoder"):
        from . import device
        return getattr(device, name)
    raise AttributeError(name)
