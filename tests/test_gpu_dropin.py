"""The SPA_Decoder drop-in, driven the way the reference's main.py drives it.

A main.py-style per-frame loop (main.py:295-342: DataBuffer -> channel ->
decoder.decode(db) -> counters) over the golden frames: decode() must return
Result.OK / DATA_TRANSFER_NOT_OK, write _decoded_data and set
convergence_iteration / _normalized_llr_by_iterations exactly as the
reference did on the same inputs.
"""
import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu


class DataBuffer:
    """The fields of python_ldpc_app/data_buffer.py:16-25 that decode() touches."""

    def __init__(self, ch):
        self._channel_data = list(map(float, ch))
        self._decoded_data = []


@pytest.mark.parametrize("set_name", ["bch_T10", "w576_T5", "bch_edge_T3"])
def test_main_loop_dropin(gpu_available, set_name):
    import ldpc_amd
    from ldpc_amd import Result, Settings, SPA_Decoder
    g = load_golden(set_name)
    code = str(g["code"])
    edd = ldpc_amd.load_committed_code(code)
    settings = Settings()
    settings.set_max_iterations(int(g["T"]))
    settings.set_normalized_llr_calculate(bool(g["nllr_on"]))
    decoder = SPA_Decoder(edd, settings)
    n_frames = min(len(g["ch"]), 64)
    hist_len = 0
    for f in range(n_frames):
        db = DataBuffer(g["ch"][f])
        res = decoder.decode(db)
        assert res == (Result.OK if g["ok"][f] else Result.DATA_TRANSFER_NOT_OK)
        assert db._decoded_data == g["z"][f].astype(int).tolist()
        assert decoder.convergence_iteration == int(g["conv"][f])
        if bool(g["nllr_on"]):
            assert decoder._d_summarize_normalized_llr == float(g["nllr"][f])
            iters = int(g["conv"][f]) + 1 if g["conv"][f] >= 0 else int(g["T"])
            hist_len += iters
            assert len(decoder._normalized_llr_by_iterations) == hist_len  # lists accumulate (:19-22)


def test_dropin_accepts_caller_result_enum(gpu_available, monkeypatch):
    """Inside the reference's main.py, decode() must return ITS enums.Result."""
    import enum
    import sys
    import types

    import ldpc_amd
    from ldpc_amd import Settings, SPA_Decoder

    class Result(enum.Enum):
        OK = "eOk"
        DATA_TRANSFER_NOT_OK = "eDataTransferNotOk"

    mod = types.ModuleType("enums")
    mod.Result = Result
    monkeypatch.setitem(sys.modules, "enums", mod)
    g = load_golden("bch_T10")
    dec = SPA_Decoder(ldpc_amd.load_committed_code("BCH_7_4_1_strip"), Settings(max_iterations=10))
    assert dec.decode(DataBuffer(g["ch"][0])) is Result.OK
