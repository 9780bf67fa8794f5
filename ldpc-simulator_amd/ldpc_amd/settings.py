"""Decoder settings mirrored from python_ldpc_app/settings.py:4-89 (the getters
SPA_Decoder.decode reads: get_max_iterations, is_normalized_llr_calculate)."""


class Settings:
    def __init__(self, max_iterations=5, normalized_llr=False):
        self._i_blocks_cnt = 100
        self._max_iterations = max_iterations  # settings.py:7 default 5
        self._b_ber_calculate = True
        self._b_fer_calculate = False
        self._b_is_calculate_normalized_llr = normalized_llr

    def set_blocks_cnt(self, n):
        self._i_blocks_cnt = n

    def get_blocks_cnt(self):
        return self._i_blocks_cnt

    def set_max_iterations(self, n):
        self._max_iterations = n

    def get_max_iterations(self):
        return self._max_iterations

    def set_ber_calculate(self, b):
        self._b_ber_calculate = b

    def is_ber_calculate(self):
        return self._b_ber_calculate

    def set_fer_calculate(self, b):
        self._b_fer_calculate = b

    def is_fer_calculate(self):
        return self._b_fer_calculate

    def set_normalized_llr_calculate(self, b):
        self._b_is_calculate_normalized_llr = b

    def is_normalized_llr_calculate(self):
        return self._b_is_calculate_normalized_llr
