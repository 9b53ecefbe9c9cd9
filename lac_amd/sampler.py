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

Per-token semantics follow the reference exactly, although the bits are coded
later: the sampler mirrors the coder's Region registers (low, high) on the host
-- the floor-mapped narrowing and renormalisation of Region.step/emit, integer
work per token -- so that ``sample_scaled_cdf`` can run the reference's
unencodable-token assertion (every token's float-mapped width at the *current*
region must be positive, :74-77) and report ``bits_per_token`` as
``Region.entropy_of`` (:155-157), both of which depend on the current span.  The
output bits come only from the GPU coder; the GPU's final registers are checked
against the mirror at flush (a mismatch raises).

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
        self._low, self._high = 0, self.one - 1         # Region registers (arithmetic_coding.py:145-147)

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

    # -- host mirror of Region (arithmetic_coding.py:128-177); registers only
    @property
    def span(self):
        return self._high - self._low + 1

    def _map(self, v, d):
        """Region.map (:158-160) on Python ints."""
        return self._low + (self.span * v) // d

    def entropy_of(self, l, h, d):
        """Region.entropy_of (:155-157)."""
        lm, hm = self._map(l, d), self._map(h, d)
        return math.log2(self.span) - math.log2(hm - lm)

    def _region_step(self, l, h, d):
        """Region.step + emit (:164-172): narrow, then renormalise (bits go to the GPU coder)."""
        low, high = self._map(l, d), self._map(h, d) - 1
        one, p = self.one, self.precision
        while (high - low + 1) * 2 <= one:
            bit = low >> (p - 1)
            low = (low << 1) - (bit << p)
            high = ((high << 1) + 1) - (bit << p)
        self._low, self._high = low, high

    def _check_encodable(self, cdf):
        """The reference's assertion (:74-77), same numpy float64 expression: every
        token's float-mapped width at the current region must be positive."""
        mapped = self._low + (self.span * cdf.astype(float)) // float(cdf[-1])
        mpdf = np.diff(np.concatenate((np.array([0]), mapped - self._low)))
        minpdf = np.min(mpdf)
        if not minpdf > 0:
            raise AssertionError(f"cdf has unencodable token {np.argmin(mpdf)} (pdf = {minpdf})."
                                 " Perhaps try using get_lop_bias or adding an arange to the cdf.")

    def sample_scaled_cdf(self, cdf):
        cdf = np.asarray(cdf)
        self._check_encodable(cdf)
        if self._compress_tokens is None:
            raise NotImplementedError("ACSampler decompression is not provided (see module docstring)")
        try:
            tok = next(self._compress_tokens)
        except StopIteration:
            self.compress_done = True
            if self.on_compress_done:
                self.on_compress_done()
            return 0
        if not (0 <= tok < len(cdf)):
            raise AssertionError(f"token {tok} outside the cdf")
        pmf = np.empty(len(cdf), dtype=np.uint64)
        pmf[0] = cdf[0]
        pmf[1:] = cdf[1:] - cdf[:-1]
        low = int(cdf[tok - 1]) if tok else 0
        high, denom = int(cdf[tok]), int(cdf[-1])
        if self.bits_per_token:
            self.bits_per_token(self.entropy_of(low, high, denom))
        self._region_step(low, high, denom)
        self._rows.append(pmf)
        self._toks.append(int(tok))
        return tok

    def flush_compress(self):
        """Code every queued token on the GPU and emit the bits (flush_compress :50-56)."""
        bits, regs = encode_acsampler(self._rows, self._toks, self.precision, registers=True)
        if self._rows and regs != (self._low, self._high):
            raise RuntimeError(f"GPU coder registers {regs} differ from the Region mirror "
                               f"{(self._low, self._high)}")
        self._rows, self._toks = [], []
        self._low, self._high = 0, self.one - 1          # Region.reset (:145-147)
        if self.compress_output:
            for b in bits:
                self.compress_output(b)


def encode_acsampler(rows, toks, prec=48, device=None, registers=False):
    """ACSampler-format bits for per-token pmf rows (uint64) and tokens, on the GPU
    (with ``registers``: also the coder's (low, high) after the last token)."""
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
    regs = None
    if registers:
        l, h = coder.registers()
        regs = (int(l[0]), int(h[0]))
    coder.finish()
    coder.raise_on_error()
    data, nb = coder.to_bytes()
    L = int(nb[0])
    coder.close()
    bits = [(data[0][i >> 3] >> (7 - (i & 7))) & 1 for i in range(L)]
    return (bits, regs) if registers else bits


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
