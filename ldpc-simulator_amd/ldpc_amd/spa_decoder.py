"""Drop-in SPA_Decoder backed by the HIP kernels (libldpc_hip.so).

Same constructor and call as python_ldpc_app/spa_decoder.py:
    SPA_Decoder(encoder_decoder_data, settings)            (:16-42)
    decode(data_buffer) -> Result                          (:63-280)
Construction does no HIP work: the graph upload and the device workspace are
made by the first decode() in the process that calls it.  It does validate H
(ldpc_graph_create's checks, HIP-free), so a malformed matrix fails in the
constructor, as in the reference; a bad device or an HBM shortfall surfaces
on the first decode().  main.py:221 builds
a decoder in the parent and then forks a ProcessPoolExecutor whose workers
build their own (main.py:78, main.py:248-256; adaptive.py:227-282): the
parent never starts HIP, each worker starts its own (ldpc_amd._lib.gpu).

decode() reads data_buffer._channel_data, writes data_buffer._decoded_data (the hard
output z, the complement of the bit estimate), and sets convergence_iteration,
_normalized_llr_by_iterations (appended per iteration, never reset -- :19-22,
:226-228) and _d_summarize_normalized_llr.  Failure to converge is
Result.DATA_TRANSFER_NOT_OK, not an exception; bad arguments raise.

`encoder_decoder_data` may be ours (ldpc_amd.code.EncoderDecoderData) or the
reference's: only `_h_sparse_cached` (else `_h_std`), `_m` and `_n` are read,
as the reference does.  `decode_batch` decodes many frames per launch.
"""
import os

import numpy as np
from scipy import sparse

from .device import Decoder, Graph, _csr_arrays, validate_csr
from .enums import caller_result_enum


def _graph_matrix(edd):
    H = getattr(edd, "_h_sparse_cached", None)
    if H is None:
        H = edd._h_std
        H = H.get_sparse_matrix() if hasattr(H, "get_sparse_matrix") else H
    return sparse.csr_matrix(H)


class SPA_Decoder:
    def __init__(self, encoder_decoder_data, settings, device=-1, max_frames=64):
        self.m_pData = encoder_decoder_data
        self.m_pSettings = settings
        self._arr_changed_by_iterations = []
        self._normalized_llr_by_iterations = []
        self._normalized_llr_by_iterations_soft = []
        self._d_summarize_normalized_llr = 0.0
        self._arr_aposteriori_llrs = []
        self.convergence_iteration = -1
        H = _graph_matrix(encoder_decoder_data)
        if H.shape != (encoder_decoder_data._m, encoder_decoder_data._n):
            raise ValueError(f"H_std shape {H.shape} != (m, n) = "
                             f"({encoder_decoder_data._m}, {encoder_decoder_data._n})")
        # fail fast, HIP-free: the graph checks of ldpc_graph_create and the
        # argument ranges (the device itself is first touched by decode())
        _, _, indptr, indices = _csr_arrays(H)
        validate_csr(H.shape[0], H.shape[1], indptr, indices)
        if int(device) < -1:
            raise ValueError(f"device index {device} < -1")
        if int(max_frames) < 1:
            raise ValueError(f"max_frames {max_frames} < 1")
        self.H_sparse = H
        self._device_index = device
        self._max_frames = max_frames
        self._graph = None
        self._dev = None
        self._pid = None
        self._Result = caller_result_enum()

    def _device(self):
        """Graph + workspace of THIS process, made on first use (no HIP in __init__)."""
        if self._dev is None or self._pid != os.getpid():
            self._graph = Graph.cached(self.H_sparse, self._device_index)
            self._dev = Decoder(self._graph, self._max_frames)
            self._pid = os.getpid()
        return self._dev

    # ------------------------------------------------------------ one frame
    def decode(self, p_data_buffer):
        T = int(self.m_pSettings.get_max_iterations())
        nllr = bool(self.m_pSettings.is_normalized_llr_calculate())
        ch = np.asarray(p_data_buffer._channel_data, dtype=np.float64)
        r = self._device().decode(ch[None, :], T, nllr=nllr, hist=nllr)
        self.convergence_iteration = int(r.conv[0])
        p_data_buffer._decoded_data = r.z[0].astype(np.int64).tolist()
        if nllr:
            k = self.m_pData._n - self.m_pData._m
            done = int(r.iters[0])
            vals = r.hist[0, :done]
            self._normalized_llr_by_iterations.extend(float(v) for v in vals)
            self._arr_changed_by_iterations.extend(int(round(v * k)) for v in vals)
            if self._normalized_llr_by_iterations:
                self._d_summarize_normalized_llr = self._normalized_llr_by_iterations[-1]
        return self._Result.OK if r.status[0] == 0 else self._Result.DATA_TRANSFER_NOT_OK

    # ------------------------------------------------------------ a batch
    def decode_batch(self, llr, max_iter=None, nllr=None, post=False, hist=False, msgs=False,
                     max_frames=None):
        """Decode [B, n] LLRs.  Returns dict(z, conv, status, iters, nllr, post, hist, msgs)."""
        T = int(self.m_pSettings.get_max_iterations() if max_iter is None else max_iter)
        nl = bool(self.m_pSettings.is_normalized_llr_calculate() if nllr is None else nllr)
        llr = np.asarray(llr, dtype=np.float64)
        B = llr.shape[0] if llr.ndim == 2 else 1
        dev = self._device()
        # a workspace for the whole batch if it fits the HBM budget, else
        # ldpc_decode_f64 runs the batch in chunks of the capacity
        want = max_frames or Decoder.fit_slots(self._graph, B)
        if want > dev.capacity:
            dev = self._dev = Decoder(self._graph, want)
        return dev.decode(llr, T, nllr=nl, post=post, hist=hist, msgs=msgs)
