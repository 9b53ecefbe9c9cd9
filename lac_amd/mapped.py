"""Coders for predictors that map symbols themselves.

A predictor that defines its own ``symbol_to_range`` / ``val_to_symbol`` (the
reference's toy ``Predictor`` subclasses such as ``ModifiedMarkov``,
/root/reference/arith_code.py:468-522, or a CDF predictor with a different
rounding) has no probability table the GPU kernels could scan: its mapping is
Python code.  ``AC`` / ``A_to_bin`` / ``A_from_bin`` hand such predictors to the
classes here, which call the predictor exactly where the reference does
(receive_symbol :169-175, decide_symbol :268-273, emit_symbol :274-283, flush
:300-317) and leave the register arithmetic -- narrowing, the emit_bit digit
loop, the encoder flush, emit_symbol's overlap check -- to liblac.so's host
functions (include/lac.h ``lac_hc_*``).  Table predictors never come here, and
nothing here stands in for the GPU: the library is required all the same.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib

_I8x64 = C.c_int8 * 64
_I64_MIN, _I64_MAX = -(1 << 63), (1 << 63) - 1


def _range(lo, hi):
    """A predictor's (lo, hi) as int64 arguments: ctypes would wrap anything wider
    silently ((1 << 64) + 5 arrives as 5), so a bound beyond int64 is refused."""
    lo, hi = int(lo), int(hi)
    for v in (lo, hi):
        if not _I64_MIN <= v <= _I64_MAX:
            raise _lib.LacError(_lib.LAC_E_ARG, f"symbol range bound {v} does not fit int64 (the host "
                                                "register functions keep registers within +-2^62)")
    return lo, hi


def _check(rc):
    if rc == _lib.LAC_OK:
        return
    if rc == _lib.LAC_E_ZERO_WIDTH:
        raise AssertionError("zero-width symbol range (the reference coder loops forever here)")
    if rc == _lib.LAC_E_DECODE_RANGE:
        raise AssertionError("predictor range does not correspond to val")
    raise _lib.LacError(rc, _lib.load().lac_last_error().decode(errors="replace"))


class MappedEncoderMixin:
    """A_to_bin over the predictor's own symbol_to_range (arith_code.py:156-246)."""

    def _mapped_init(self, predictor, prec):
        self._lib = _lib.load()
        self.predictor = predictor
        self.precision = prec
        self.denom = 1 << prec
        self.decision = 1 << (prec - 1)
        self._l, self._h = 0, self.denom - 1
        self.emitted_bits = 0
        self.debug_log = None

    @property
    def l(self):
        return self._l

    @property
    def h(self):
        return self._h

    def _log_emits(self, digits):
        l, h = self._l, self._h
        for d in digits:
            self.debug_log.append((l, h, "emit", d))
            l, h = l * 2 - d * self.denom, h * 2 + 1 - d * self.denom

    def step(self, symbol):
        if self.debug_log:
            self.debug_log.append((self._l, self._h, "recv", symbol))
        lo, hi = _range(*self.predictor.symbol_to_range(symbol, self._h - self._l + 1))
        l, h = C.c_int64(self._l), C.c_int64(self._h)
        dig, n = _I8x64(), C.c_int32()
        _check(self._lib.lac_hc_encode_symbol(self.precision, C.byref(l), C.byref(h), lo, hi, dig, C.byref(n)))
        digits = list(dig[:n.value])
        if self.debug_log:
            self._l, self._h = self._l + lo, self._l + hi - 1
            self._log_emits(digits)
        self._l, self._h = l.value, h.value
        self.predictor.accept(symbol)
        self.emitted_bits += len(digits)
        yield from digits

    def flush(self):
        dig, n = _I8x64(), C.c_int32()
        _check(self._lib.lac_hc_encode_flush(self.precision, self._l, self._h, dig, C.byref(n)))
        digits = list(dig[:n.value])
        if self.debug_log:
            self._log_emits(digits)
        self.emitted_bits += len(digits)
        self._l, self._h = 0, self.denom - 1
        yield from digits

    def run(self, symbols, stop=1):
        for s in symbols:
            yield from self.step(s)
        if stop:
            yield from self.flush()


class MappedDecoderMixin:
    """A_from_bin over the predictor's own val_to_symbol / symbol_to_range
    (arith_code.py:248-334), bit-serial as the reference."""

    def _mapped_init(self, predictor, prec):
        self._lib = _lib.load()
        self.predictor = predictor
        self.precision = prec
        self.denom = 1 << prec
        self.decision = 1 << (prec - 1)
        self._fresh()

    def _fresh(self):
        self._r = np.array([0, self.denom - 1, 0, self.denom - 1], dtype=np.int64)   # l, h, lb, hb

    def _regs(self):
        return tuple(int(v) for v in self._r)

    def _emit(self, s, renormalise):
        l, h = int(self._r[0]), int(self._r[1])
        lo, hi = _range(*self.predictor.symbol_to_range(s, h - l + 1))
        _check(self._lib.lac_hc_decode_emit(self.precision, self._r.ctypes.data_as(C.c_void_p), lo, hi,
                                            int(renormalise)))
        self.predictor.accept(s)
        return s

    def step(self, bit):
        bit = int(bit)
        if bit not in (0, 1):
            raise ValueError("bits are 0 or 1")
        return self._step(bit)

    def _step(self, bit):
        l, h, lb, hb = self._regs()                    # receive_bit, :264-267
        half = (hb - lb + 1) // 2
        self._r[2] = lb + half * bit
        self._r[3] = int(self._r[2]) + half - 1
        while True:                                    # decide_symbol, :268-273
            l, h, lb, hb = self._regs()
            w = h - l + 1
            s = self.predictor.val_to_symbol(lb - l, w)
            if s != self.predictor.val_to_symbol(hb - l, w):
                return
            yield self._emit(s, True)

    def flush(self):
        def ratio(s):                                  # the reference's k(s), :305-307
            l, h, lb, hb = self._regs()
            lo, hi = self.predictor.symbol_to_range(s, h - l + 1)
            return max(0, min(hi - 1, hb - l) - max(lo, lb - l) + 1) / (hi - lo)
        still = 0
        while True:
            l, h, lb, hb = self._regs()
            if lb <= l and h <= hb:
                break
            w = h - l + 1
            ls = self.predictor.val_to_symbol(lb - l, w)
            hs = self.predictor.val_to_symbol(hb - l, w)
            yield self._emit(max(range(ls, hs + 1), key=ratio), False)
            still = still + 1 if self._regs()[:2] == (l, h) else 0
            if still >= 1000:                          # a full-range symbol: the reference loops forever
                raise RuntimeError("A_from_bin.flush does not terminate here (the reference loops forever, "
                                   "arith_code.py:308-313)")
        self._fresh()

    def _run(self, bits, stop, max_symbols=None):
        for b in bits:
            yield from self.step(b)
        if stop:
            yield from self.flush()

    def run(self, bits, stop=1, n=None, max_symbols=None):
        if n is None:
            return self._run(bits, stop)
        out = []
        bl = [int(b) for b in bits]
        i = 0
        while len(out) < n and i < len(bl) + 4 * (n + 1) * self.precision:
            out.extend(self.step(bl[i] if i < len(bl) else 0))
            i += 1
        if len(out) < n:
            raise AssertionError("predictor range does not correspond to val")
        return iter(out[:n])
