"""Boundary types mirrored from python_ldpc_app/enums.py:4-25."""
import sys
from enum import Enum


class Result(Enum):
    OK = "eOk"
    INVALID_INPUT = "eInvalidInput"
    INVALID_PATH = "eInvalidPath"
    DATA_TRANSFER_NOT_OK = "eDataTransferNotOk"


class LDPCDecoderType(Enum):
    BIT_FLIPPING = "eBitFlipping"
    SUM_PRODUCT = "eSumProduct"


def caller_result_enum():
    """The Result enum the caller compares against.

    When this decoder is dropped into the reference's main.py, `decode()` must
    return the caller's own `enums.Result` members (main.py:314 compares
    `result == Result.OK`).  If a module named `enums` with a compatible
    `Result` is loaded, use it; otherwise use ours.
    """
    mod = sys.modules.get("enums")
    res = getattr(mod, "Result", None) if mod is not None else None
    if res is not None and hasattr(res, "OK") and hasattr(res, "DATA_TRANSFER_NOT_OK"):
        return res
    return Result
