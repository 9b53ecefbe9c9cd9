"""ACSampler (encode side) on the GPU coder -- /root/reference/arithmetic_coding.py.

The reference's second coder is a *sampler*: the model loop calls
``sample(pdf)`` once per token; while compressing, the sampler takes the next
token from ``compress_tokens``, codes it and returns it (:57-124).  This class
keeps that loop and its callbacks (``compress_tokens``, ``compress_output``,
``on_compress_done``, ``bits_per_token``), and quantises each float pdf to the
same uint64 CDF with the same numpy float64 operations in the same order
(``sample`` :57-62, ``get_lop_bias`` :63-72): that is the model-side
quantiser, not the coder.

The coder -- Region.map/step/emit (:160-177, floor mapping), CarryBuffer
(:180-208) and flush_compress (:50-56) -- runs on the GPU through liblac.so
(LAC_MAP_FLOOR + LAC_TERM_ACSAMPLER).  Because a token's output bits are final
only at flush time anyway, rows are queued and coded in one launch when the
tokens run out; ``compress_output`` then receives every output bit in order, the
same bit sequence the reference emits incrementally.

Decompression is not provided: the reference's decoder is broken under
numpy >= 2 and mis-decodes ~45% of streams even with exact CDFs (SURVEY.md
finding 4); use lac_amd.coder / lac_amd.batch (A_to_bin format) instead.
"""
from __future__ import annotations

import math

import numpy as np

from .batch import BatchCoder


class ACSampler:
    def __init__(self, precision=48):
        self.precision = precision
        self.one = 1 << precision
        self.compress_tokens = None
        self.compress_output = None
        self.bits_per_token = None
        self.on_compress_done = None
        self.compress_done = False
        self._rows = []
        self._toks = []
        self._span_bits = 0.0

    @property
    def compress_tokens(self):
        return self._compress_tokens

    @compress_tokens.setter
    def compress_tokens(self, toks):
        self._compress_tokens = iter(toks) if toks is not None else None
        self.compress_done = False

    def get_lop_bias(self, pdf):
        """arithmetic_coding.py:63-72 (builtin sum, as the reference)."""
        return sum(pdf) / (self.one / 2 - len(pdf))

    def quantise(self, pdf):
        """float pdf -> the reference's uint64 CDF (arithmetic_coding.py:58-61)."""
        pdf = np.array(pdf, dtype=np.float64)
        pdf += self.get_lop_bias(pdf)
        pdf *= self.one / np.sum(pdf)
        return np.cumsum(pdf).astype(np.uint64)

    def sample(self, pdf):
        return self.sample_scaled_cdf(self.quantise(pdf))

    def sample_scaled_cdf(self, cdf):
        if self._compress_tokens is None:
            raise NotImplementedError("ACSampler decompression is not provided (see module docstring)")
        try:
            tok = next(self._compress_tokens)
        except StopIteration:
            self.compress_done = True
            if self.on_compress_done:
                self.on_compress_done()
            return 0
        pmf = np.empty(len(cdf), dtype=np.uint64)
        pmf[0] = cdf[0]
        pmf[1:] = cdf[1:] - cdf[:-1]
        if not (0 <= tok < len(cdf)) or pmf[tok] == 0:
            raise AssertionError(f"cdf has unencodable token {tok}")
        if self.bits_per_token:
            self.bits_per_token(math.log2(float(cdf[-1])) - math.log2(float(pmf[tok])))
        self._rows.append(pmf)
        self._toks.append(int(tok))
        return tok

    def flush_compress(self):
        """Code every queued token on the GPU and emit the bits (flush_compress :50-56)."""
        bits = encode_acsampler(self._rows, self._toks, self.precision)
        self._rows, self._toks = [], []
        if self.compress_output:
            for b in bits:
                self.compress_output(b)


def encode_acsampler(rows, toks, prec=48, device=None):
    """ACSampler-format bits for per-token pmf rows (uint64) and tokens, on the GPU."""
    import torch
    n = len(toks)
    V = len(rows[0]) if rows else 1
    static = all(r is rows[0] or np.array_equal(r, rows[0]) for r in rows[1:]) if rows else True
    coder = BatchCoder(V, 1, prec=prec, pmf_bits=64, capacity_bits=(n + 2) * (prec + 2) + 256, device=device)
    coder.set_mapping("floor")
    coder.set_termination("acsampler")
    if rows:
        tab = np.asarray(rows[0] if static else np.stack(rows), dtype=np.uint64)
        pmf = torch.from_numpy(tab.view(np.int64).copy()).to(coder.device)
        sym = torch.tensor(toks, dtype=torch.int32, device=coder.device).view(n, 1)
        coder.encode(pmf if static else pmf.view(n, 1, V), sym)
    coder.finish()
    coder.raise_on_error()
    data, nb = coder.to_bytes()
    L = int(nb[0])
    coder.close()
    return [(data[0][i >> 3] >> (7 - (i & 7))) & 1 for i in range(L)]


class packbits:
    """MSB-first bit -> byte packer with zero-padding flush (arithmetic_coding.py:212-225)."""

    def __init__(self, byte_callback):
        self.state = 1
        self.byte_callback = byte_callback

    def __call__(self, bit):
        self.state <<= 1
        self.state |= bit
        if self.state >> 8:
            self.byte_callback(self.state & 255)
            self.state >>= 8

    def flush(self):
        while self.state > 1:
            self(0)


def unpackbits(byte_generator):
    """arithmetic_coding.py:227-230."""
    for byte in byte_generator:
        for b in range(8):
            yield (byte >> (7 - b)) & 1
