"""Channels (mirror of channels.py:4-26, plus BSC and BI-AWGN).

Host methods keep the reference's numpy behaviour for per-trial callers;
``device_outputs`` generates a whole batch on the MI355X (Philox4x32-10,
counter = (codeword, variable), see ldpc_channel_dev) so Monte-Carlo never
round-trips channel noise through the host.
"""
import numpy as np

from . import decoder
from ._native import CH_AWGN, CH_BEC, CH_BSC


class BEC:
    """Binary erasure channel.  Bit mappings as channels.py:5: 0 -> -1, ? -> 0, 1 -> 1
    for ``transmit``; ``new_transmit`` keeps 0/1 and marks erasures 2."""
    kind = CH_BEC

    def __init__(self, erasure_prob):
        self.erasure_prob = erasure_prob

    @property
    def param(self):
        return self.erasure_prob

    def transmit(self, input_binary):  # channels.py:19-22
        input_binary = np.where(input_binary == 0, -1, input_binary)
        random_vector = np.random.rand(len(input_binary))
        return np.where(random_vector < self.erasure_prob, 0, input_binary)

    def new_transmit(self, input_binary):  # channels.py:24-26
        random_vector = np.random.rand(len(input_binary))
        return np.where(random_vector < self.erasure_prob, 2, input_binary)

    def device_outputs(self, seed, first_cw, n, B, out=None):
        return decoder.channel_dev(CH_BEC, self.erasure_prob, seed, first_cw, n, B, out)


class BSC:
    """Binary symmetric channel, crossover p; outputs LLRs +-ln((1-p)/p)."""
    kind = CH_BSC

    def __init__(self, crossover_prob):
        self.crossover_prob = crossover_prob

    @property
    def param(self):
        return self.crossover_prob

    def llr_magnitude(self):
        return float(np.float32(np.log((1.0 - self.crossover_prob) / self.crossover_prob)))

    def transmit(self, input_binary):
        flips = np.random.rand(len(input_binary)) < self.crossover_prob
        return np.bitwise_xor(np.asarray(input_binary, dtype=np.int64), flips.astype(np.int64))

    def llr(self, received):
        lc = self.llr_magnitude()
        return np.where(np.asarray(received) == 1, -lc, lc).astype(np.float32)

    def device_outputs(self, seed, first_cw, n, B, out=None):
        return decoder.channel_dev(CH_BSC, self.crossover_prob, seed, first_cw, n, B, out)


class BIAWGN:
    """Binary-input AWGN: BPSK 0 -> +1, 1 -> -1, noise std sigma, LLR = 2y/sigma^2."""
    kind = CH_AWGN

    def __init__(self, sigma):
        self.sigma = sigma

    @property
    def param(self):
        return self.sigma

    @classmethod
    def from_ebn0_db(cls, ebn0_db, rate):
        return cls(float(np.sqrt(1.0 / (2.0 * rate * 10.0 ** (ebn0_db / 10.0)))))

    def transmit(self, input_binary):
        x = 1.0 - 2.0 * np.asarray(input_binary, dtype=np.float64)
        return x + self.sigma * np.random.randn(len(x))

    def llr(self, y):
        return (2.0 / self.sigma ** 2 * np.asarray(y)).astype(np.float32)

    def device_outputs(self, seed, first_cw, n, B, out=None):
        return decoder.channel_dev(CH_AWGN, self.sigma, seed, first_cw, n, B, out)
