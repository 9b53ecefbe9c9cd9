"""The reference's predictor -> coder surface, running on the GPU coder.

Drop-in counterparts of /root/reference/arith_code.py:

    region_overlap          :59-61
    Predictor               :64-74   (uniform n-ary; floor mapping)
    CDFPredictor            :76-110  (CDF table; ceil mapping; fudged_dist)
    ProbPredictor           :111-135 (prob / calc_dist / cached dist)
    AC                      :144-155 (.to_bin / .from_bin make fresh coders)
    A_to_bin                :156-246 (step, run, bits, encode, flush, __call__)
    A_from_bin              :248-334 (step, run, decode)
    group_bits/ungroup_bits :336-351
    measure_compress        :401-420

The predictor classes keep the reference's arithmetic so that third-party
subclasses (History, Markov, an LLM adapter overriding ``calc_dist``) keep
working, but the coders never call ``symbol_to_range``/``val_to_symbol``: they
hand each step's integer pmf row (from ``predictor.dist``) to liblac.so, whose
kernels implement exactly that arithmetic on the device.  A ``Predictor`` that
is not table-based (custom ``symbol_to_range`` with no ``dist``) is rejected with
TypeError: there is no CPU coder behind this API.

Coding one symbol at a time through ``step`` is correct but launch-bound; use
``run``/``bits``/``encode`` (one launch for the whole sequence) or the batched
``lac_amd.batch.BatchCoder`` for throughput.
"""
from __future__ import annotations

import bisect
import itertools
import math

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check
from .batch import BatchCoder, digits_of


def region_overlap(a, b, c, d):
    """[a,b] with [c,d] (closed intervals) -- arith_code.py:59-61."""
    return max(0, min(d, b) - max(a, c) + 1)


# ------------------------------------------------------------------ predictors
class Predictor:
    """Uniform n-ary predictor (arith_code.py:64-74)."""

    def __init__(self, n):
        self.n = n

    def val_to_symbol(self, v, denom):
        return (v * self.n) // denom

    def symbol_to_range(self, s, denom):
        return (s * denom) // self.n, ((s + 1) * denom) // self.n

    def accept(self, symbol):
        pass

    def copy(self):
        return self


class CDFPredictor(Predictor):
    """CDF-table predictor (arith_code.py:76-110).  ``dist`` is the inclusive CDF."""

    def __init__(self, dist):
        self.dist = dist
        self.minp = min(filter(lambda v: v > 0, self.pdf_iter))

    @property
    def pdf_iter(self):
        d = self.dist
        return itertools.chain([d[0]], (d[i + 1] - d[i] for i in range(len(d) - 1)))

    def fudged_dist(self, denom):
        if self.dist[-1] <= denom * self.minp:
            return self.dist
        res = []
        p = 0
        n = len(self.dist)
        for i in range(n):
            d = (int(self.dist[i]) * denom) // int(self.dist[-1]) - p
            d = max(1, min(denom - p - n + i + 1, d))
            p += d
            res.append(p)
        return res

    def val_to_symbol(self, v, denom):
        dist = self.fudged_dist(denom)
        return bisect.bisect_right(dist, (v * int(dist[-1])) // denom)

    def symbol_to_range(self, s, denom):
        dist = self.fudged_dist(denom)
        if s >= len(dist) or s < 0:
            raise AssertionError("unknown symbol", s)
        hd = int(dist[s])
        ld = int(dist[s - 1]) if s > 0 else 0
        d = int(dist[-1])
        return -(-(ld * denom) // d), -(-(hd * denom) // d)


class ProbPredictor(CDFPredictor):
    """Probability-vector predictor (arith_code.py:111-135): override ``prob`` or
    ``calc_dist`` (an LLM adapter returns its quantised CDF there)."""

    def __init__(self, n):
        self.n = n
        self.dcache = None

    def prob(self, symbol):
        return 1

    def calc_dist(self):
        p = 0
        self.dcache = []
        for s in range(self.n):
            p += self.prob(s)
            self.dcache.append(p)
        return self.dcache

    @property
    def dist(self):
        if self.dcache is None:
            return self.calc_dist()
        return self.dcache

    @property
    def minp(self):
        return min(filter(lambda v: v > 0, self.pdf_iter))

    def accept(self, symbol):
        self.dcache = None

    def copy(self):
        return self


ternary = Predictor(3)


# ------------------------------------------------------------------ tables
def _row_of(predictor):
    """The predictor's current integer pmf row (numpy uint64) from its CDF."""
    fast = getattr(predictor, "pmf_row", None)
    if fast is not None:
        return np.asarray(fast(), dtype=np.uint64)
    d = getattr(predictor, "dist", None)
    if d is None:
        raise TypeError(f"{type(predictor).__name__} exposes no probability table (.dist); the GPU coder "
                        "needs CDFPredictor/ProbPredictor-style predictors")
    cdf = np.asarray([int(x) for x in d], dtype=object) if not isinstance(d, np.ndarray) or d.dtype == object \
        else d.astype(object)
    pmf = np.empty(len(cdf), dtype=object)
    pmf[0] = int(cdf[0])
    pmf[1:] = cdf[1:] - cdf[:-1]
    if any(int(x) < 0 for x in pmf):
        raise ValueError("dist is not monotone non-decreasing")
    return np.array([int(x) for x in pmf], dtype=np.uint64)


def _is_uniform(predictor):
    """A table-less Predictor(n) with the base class's floor mapping (arith_code.py:64-74)."""
    if getattr(predictor, "dist", None) is not None or not hasattr(predictor, "n"):
        return False
    stv = getattr(type(predictor), "symbol_to_range", None)
    return stv is Predictor.symbol_to_range or (type(predictor).__name__ == "Predictor"
                                                 and type(predictor).__module__ != __name__)


def _raise_for(code, sym=None):
    if code == _lib.LAC_E_SYMBOL_RANGE:
        raise AssertionError("unknown symbol", sym)
    if code == _lib.LAC_E_DECODE_RANGE:
        raise AssertionError("predictor range does not correspond to val")
    if code == _lib.LAC_E_ZERO_WIDTH:
        raise AssertionError("zero-probability symbol (the reference coder loops forever here)", sym)
    raise _lib.LacError(code, "coder error")


class _Tables:
    """Per-step rows from a predictor.  A uniform Predictor(n) becomes a row of n
    ones coded with the floor mapping (Predictor.symbol_to_range, :69-70)."""

    def __init__(self, predictor):
        self.p = predictor
        self.uniform = _is_uniform(predictor)
        self.mapping = "floor" if self.uniform else "ceil"

    def row(self):
        if self.uniform:
            return np.ones(int(self.p.n), dtype=np.uint64)
        return _row_of(self.p)


# ------------------------------------------------------------------ encoder
class A_to_bin:
    """Encoder (arith_code.py:156-246) backed by liblac.so (one stream)."""

    def __init__(self, predictor=ternary, prec=16):
        self.predictor = predictor
        self.precision = prec
        self.denom = 1 << prec
        self.decision = 1 << (prec - 1)
        self.emitted_bits = 0
        self.debug_log = None
        self._coder = None
        self._V = None
        self._plane_bits = 0          # output bits held in the device planes since the last reset
        self._nsym = 0                # symbols coded since the last reset

    # -- device plumbing
    # Digits reach the caller through the per-symbol trace, so the device's own
    # output planes only have to hold what was coded since the last reset (or
    # rebase, which keeps the registers and drops finished words): a stream of
    # any length -- step() loops, repeated run() calls, reuse after flush() --
    # fits a fixed capacity.
    _SLACK = 256                      # flush digits + the word a rebase keeps

    def _ensure(self, V, steps):
        per = self.precision + 1      # one symbol emits at most prec digits (renorm)
        need = (steps + 2) * per + self._SLACK
        if self._coder is not None and self._V == V:
            return
        if self._coder is not None and self._plane_bits:
            raise RuntimeError(f"table size changed mid-stream ({self._V} -> {V} symbols); flush() first")
        if self._coder is not None:
            self._coder.close()
        self._coder = BatchCoder(V, 1, prec=self.precision, pmf_bits=64, capacity_bits=max(need * 2, 1 << 12))
        self._coder.set_mapping(_Tables(self.predictor).mapping)
        self._V = V
        self._plane_bits = 0
        self._nsym = 0

    def _encode_rows(self, rows, syms):
        """Encode rows/syms (chunked to the coder's capacity); -> (digit lists, (rc, n_ok))."""
        steps = len(syms)
        V = len(rows[0])
        if self._coder is not None and self._V == V and self._plane_bits == 0:
            per = self.precision + 1
            if self._coder.capacity_bits < (steps + 2) * per + self._SLACK:
                self._coder.close()
                self._coder = None    # empty planes: reallocate at the new size
        self._ensure(V, steps)
        per = self.precision + 1
        out = []
        i = 0
        while i < steps:
            room = (self._coder.capacity_bits - self._plane_bits - self._SLACK) // per
            if room < 1:
                self._coder.rebase()
                self._plane_bits = 64
                continue
            n = min(room, steps - i)
            digs, rc, n_ok = self._encode_chunk(rows[i:i + n], syms[i:i + n])
            out.extend(digs)
            if rc:
                return out, (rc, i + n_ok)
            i += n
        return out, (0, steps)

    def _encode_chunk(self, rows, syms):
        import torch
        steps = len(syms)
        V = len(rows[0])
        dev = self._coder.device
        pmf = torch.from_numpy(np.stack(rows).astype(np.uint64).view(np.int64).reshape(steps, 1, V)).to(dev)
        sym = torch.tensor([int(s) if 0 <= int(s) < 2 ** 31 else -1 for s in syms], dtype=torch.int32,
                           device=dev).view(steps, 1)
        tr = torch.zeros((steps, 1, 2), dtype=torch.int64, device=dev)
        self._coder.encode(pmf, sym, trace=tr)
        rc, err, step = self._coder.status()
        t = tr.cpu().numpy()
        # err_step counts symbols since the last reset: the failing one's index in this chunk
        n_ok = steps if rc == 0 else min(max(int(step[0]) - self._nsym, 0), steps)
        self._nsym += n_ok
        digs = [digits_of(int(E), int(k)) for E, k in t[:n_ok, 0]]
        for d in digs:
            self.emitted_bits += len(d)
            self._plane_bits += len(d)
        return digs, rc, n_ok

    # -- registers (reference attributes)
    @property
    def l(self):
        return int(self._coder.registers()[0][0]) if self._coder else 0

    @property
    def h(self):
        return int(self._coder.registers()[1][0]) if self._coder else self.denom - 1

    def __repr__(self):
        sl = bin(self.l + (self.denom << 1))[3:]
        sh = bin(self.h + (self.denom << 1))[3:]
        return f"A_to_bin([{sl[0]}.{sl[1:]},{sh[0]}.{sh[1:]}])"

    # -- reference API
    def step(self, symbol):
        tab = _Tables(self.predictor)
        row = tab.row()
        digs, (rc, n_ok) = self._encode_rows([row], [symbol])
        if rc:
            _raise_for(rc, symbol)
        self.predictor.accept(symbol)
        yield from digs[0]

    def __call__(self, symbol):
        if symbol is None:
            return tuple(self.flush())
        return tuple(self.step(symbol))

    def flush(self):
        if self._coder is None:
            tab = _Tables(self.predictor)
            self._ensure(len(tab.row()), 0)
        self._coder.finish()
        rc, err, step = self._coder.status()
        if rc:
            _raise_for(rc)
        fd = self._coder.flush_digits()[0]
        self.emitted_bits += len(fd)
        yield from fd
        self._coder.reset()
        self._plane_bits = 0
        self._nsym = 0

    def _collect(self, symbols):
        tab = _Tables(self.predictor)
        rows, syms = [], []
        for s in symbols:
            rows.append(tab.row())
            syms.append(s)
            if not (0 <= int(s) < len(rows[-1])):
                break                                   # the reference raises at this symbol
            self.predictor.accept(s)
        return rows, syms

    def run(self, symbols, stop=1):
        rows, syms = self._collect(symbols)
        if syms:
            digs, (rc, n_ok) = self._encode_rows(rows, syms)
            for d in digs:
                yield from d
            if rc:
                _raise_for(rc, syms[n_ok])
        if stop:
            yield from self.flush()

    def encode(self, symbols, stop=1):
        r = 0
        length = 0
        for v in self.run(symbols, stop):
            r = (r << 1) + v
            length += 1
        return r, length

    @property
    def info(self):
        return -math.log2((self.h - self.l + 1) / self.denom)

    @property
    def total_encoded_entropy(self):
        return self.emitted_bits + self.info

    @property
    def certain(self):
        return 0 <= self.l and self.h < self.denom

    def bits(self, symbols, stop=1):
        """Output bits (binary of sum d_k 2^(L-1-k), exactly L of them)."""
        r, L = self.encode(symbols, stop)
        for k in range(L - 1, -1, -1):
            yield (r >> k) & 1


# ------------------------------------------------------------------ decoder
class A_from_bin:
    """Decoder (arith_code.py:248-334) backed by liblac.so (one stream).

    The reference decodes bit-serially and stops when the bits run out; the
    stream itself does not record its symbol count (SURVEY.md finding 5), so
    ``run``/``decode`` take ``n``, the number of symbols to produce.
    """

    def __init__(self, predictor=ternary, prec=16):
        self.predictor = predictor
        self.precision = prec
        self.denom = 1 << prec
        self.decision = 1 << (prec - 1)

    def run(self, bits, stop=1, n=None, max_symbols=1 << 24):
        """Decode ``bits`` (an iterable of 0/1).

        With ``n`` given: exactly n symbols (reads zero bits past the end).
        Without: every symbol the bits determine -- the count the reference's
        bit-serial ``run(bits, stop=0)`` emits (arith_code.py:268-299, 322-326).
        ``stop=1`` does not run the reference's heuristic flush (:300-317),
        which raises on about a fifth of valid streams (SURVEY.md finding 5).
        """
        if hasattr(self, "_sbits") and n is None:
            # bits already fed through step(): the reference's run is step() over each
            # bit (arith_code.py:322-326), continuing from where those left off
            return iter([s for b in bits for s in self._step_bit(int(b))])
        bl = [int(b) for b in bits]
        data = bytes(group_bits(iter(bl)))
        return iter(self._decode_bytes(data, len(bl), n, max_symbols))

    # ---- registers (arith_code.py:249-263): l, h and the received-bit interval [lb, hb]
    # in the same frame; bit-serial decoding keeps them on the host between bits
    @property
    def l(self):
        return int(self._sstate["l"][0]) if hasattr(self, "_sstate") else 0

    @property
    def h(self):
        return int(self._sstate["h"][0]) if hasattr(self, "_sstate") else self.denom - 1

    def _pad(self):
        if not hasattr(self, "_sstate"):
            return self.precision
        past = int(self._sstate["pos"][0]) - len(self._sbits)
        return min(max(past, 0), self.precision)

    @property
    def lb(self):
        return int(self._sstate["x"][0]) if hasattr(self, "_sstate") else 0

    @property
    def hb(self):
        return self.lb + (1 << self._pad()) - 1

    def __repr__(self):
        sl = bin(self.l + (self.denom << 1))[3:]
        sh = bin(self.h + (self.denom << 1))[3:]
        slb = bin(self.lb + (self.denom << 1))[3:]
        shb = bin(self.hb + (self.denom << 1))[3:]
        slb = "".join(slb[i] for i in range(len(slb)) if slb[i] == shb[i])
        return f"A_from_bin([{sl[0]}.{sl[1:]},{sh[0]}.{sh[1:]}],{slb[0]}.{slb[1:]})"

    # ---- bit-serial decoding: step(bit) / __call__(bit) (arith_code.py:291-298, 318-321)
    _DEC_STATE = np.dtype([("l", "<i8"), ("h", "<i8"), ("x", "<i8"), ("pos", "<u8"), ("nsym", "<i8"),
                           ("err", "<i4"), ("det", "<i4"), ("err_step", "<i8"), ("ndet", "<i8")])   # lac_dec_state

    def step(self, bit):
        """receive_bit + the decide_symbol / emit_symbol loop (arith_code.py:291-298):
        yields, once each, the symbols that the bits received so far determine --
        the same symbols after the same bits as the reference.

        The GPU decodes; between calls the decoder's registers wait on the host
        (include/lac.h lac_decode_get_state / set_state).  Each call tries the next
        symbol against the bits so far, zero-padded: when both the 0- and 1-padded
        ends of the available bits map to one symbol (the reference's ls == hs)
        it is committed, the predictor accepts it and the next is tried; otherwise
        the registers stay as they were.  A new bit inside the value window of
        the committed registers is added to x where it sits (it was read as 0)."""
        return iter(self._step_bit(int(bit)))

    def __call__(self, bit):
        if bit is None:
            raise NotImplementedError("A_from_bin.flush (arith_code.py:300-317) is not provided: its heuristic "
                                      "raises on about a fifth of valid streams (SURVEY.md finding 5)")
        return tuple(self.step(bit))

    def _step_bit(self, bit):
        import torch
        if bit not in (0, 1):
            raise ValueError("bits are 0 or 1")
        if not hasattr(self, "_sbits"):
            self._sbits = []
            self._stab = _Tables(self.predictor)
            self._scoder = None
            self._sstate = np.zeros(1, dtype=self._DEC_STATE)
            self._sstate["h"] = self.denom - 1
            self._sstate["pos"] = self.precision
            self._sstate["det"] = 1
            self._sstate["err_step"] = -1
            self._sbuf = np.zeros(64, dtype=np.uint8)        # packed bits, MSB first (host copy)
            self._sdev = None                                # its device copy, re-sent when it grows
        if (len(self._sbits) >> 3) + 8 >= len(self._sbuf):
            self._sbuf = np.concatenate([self._sbuf, np.zeros(len(self._sbuf), dtype=np.uint8)])
            self._sdev = None
        n = len(self._sbits)
        self._sbits.append(bit)
        if bit:
            self._sbuf[n >> 3] |= 0x80 >> (n & 7)
        st = self._sstate
        pos = int(st["pos"][0])
        if bit and pos - self.precision <= n < pos:          # was read as a padding 0
            st["x"] += 1 << (pos - 1 - n)
        out = []
        while True:
            row = self._stab.row()
            V = len(row)
            if self._scoder is None or self._scoder.vocab != V:
                if self._scoder is not None:
                    self._scoder.close()
                self._scoder = BatchCoder(V, 1, prec=self.precision, pmf_bits=64, capacity_bits=64)
                self._scoder.set_mapping(self._stab.mapping)
            c = self._scoder
            nb = len(self._sbits)
            if self._sdev is None or self._sdev.device != c.device:
                self._sdev = torch.from_numpy(self._sbuf.reshape(1, -1)).to(c.device)
                self._snb = torch.zeros(1, dtype=torch.int64, device=c.device)
            else:                                        # only the byte the new bit went into
                self._sdev[0, n >> 3] = int(self._sbuf[n >> 3])
            self._snb.fill_(nb)
            c.decode_open(self._sdev, self._snb)
            trial = st.copy()
            trial["det"] = 1
            trial["ndet"] = 0
            check(c.lib.lac_decode_set_state(c.ctx, trial.ctypes.data_as(C.c_void_p), c._stream))
            pmf = torch.from_numpy(row.view(np.int64).reshape(1, 1, V)).to(c.device)
            s = int(c.decode(pmf).cpu()[0, 0])
            new = np.zeros(1, dtype=self._DEC_STATE)
            check(c.lib.lac_decode_get_state(c.ctx, new.ctypes.data_as(C.c_void_p), c._stream))
            # not determined by the bits so far -- or not decodable from them yet: the
            # 0-padded window can fall below l (the reference's lb - l < 0 then maps
            # the two ends to different symbols and it emits nothing either)
            if int(new["err"][0]) or int(new["ndet"][0]) != 1:
                break
            st = new
            out.append(s)
            self.predictor.accept(s)
        self._sstate = st
        return out

    def decode(self, bits, length, stop=1, n=None):
        """A_from_bin.decode(int, length) -- arith_code.py:327-334."""
        bl = [(bits >> (length - 1 - i)) & 1 for i in range(length)]
        return self.run(bl, stop, n)

    def _decode_bytes(self, data, nbits, n, max_symbols=1 << 24):
        import torch
        tab = _Tables(self.predictor)
        out = []
        coder = None
        limit = n if n is not None else max_symbols
        for i in range(limit):
            row = tab.row()
            V = len(row)
            if coder is None:
                coder = BatchCoder(V, 1, prec=self.precision, pmf_bits=64, capacity_bits=max(nbits, 64) + 64)
                coder.set_mapping(tab.mapping)
                stride = ((len(data) + 7) // 8 + 1) * 8
                buf = np.zeros((1, stride), dtype=np.uint8)
                buf[0, :len(data)] = np.frombuffer(data, dtype=np.uint8)
                self._bits = torch.from_numpy(buf).to(coder.device)
                self._nbits = torch.tensor([nbits], dtype=torch.int64, device=coder.device)
                coder.decode_open(self._bits, self._nbits)
            pmf = torch.from_numpy(row.view(np.int64).reshape(1, 1, V)).to(coder.device)
            s = int(coder.decode(pmf).cpu()[0, 0])
            if s < 0:
                rc, err, step = coder.status()
                if n is None:
                    break
                _raise_for(int(err[0]) or _lib.LAC_E_DECODE_RANGE)
            if n is None and int(coder.determined()[0]) <= i:
                break                                   # the bits do not determine symbol i
            out.append(s)
            self.predictor.accept(s)
        if coder is not None:
            coder.close()
        return out


class AC:
    """AC(predictor, prec) -- arith_code.py:144-155."""

    def __init__(self, predictor=ternary, prec=16):
        self.predictor = predictor
        self.precision = prec

    def __repr__(self):
        return f"AC({repr(self.predictor)} at {self.precision} bits)"

    @property
    def to_bin(self):
        return A_to_bin(self.predictor.copy(), self.precision)

    @property
    def from_bin(self):
        return A_from_bin(self.predictor.copy(), self.precision)


# ------------------------------------------------------------------ bit I/O
def group_bits(bits, b=8):
    """MSB-first grouping, last group zero padded -- arith_code.py:336-347."""
    r = 1
    for v in bits:
        r <<= 1
        r |= v
        if r >> b:
            yield r ^ (1 << b)
            r >>= b
    if r > 1:
        while r >> b == 0:
            r <<= 1
        yield r ^ (1 << b)


def ungroup_bits(groups, b=8):
    """arith_code.py:348-351."""
    for g in groups:
        for i in range(b):
            yield (g >> (b - i - 1)) & 1


def measure_compress(comp, inp, print_every_out=100, print_every_inp=100, save_bits=None, inp_cb=lambda t: ""):
    """bytes(group_bits(comp.bits(inp))) -- arith_code.py:401-420 (one GPU launch)."""
    if save_bits is None:
        save_bits = []
    syms = list(inp)
    bits = list(comp.bits(iter(syms)))
    save_bits.extend(bits)
    if syms and print_every_inp:
        info = comp.total_encoded_entropy
        print(len(syms), "->", info, "   ", info / len(syms), " bits/tok ", inp_cb(syms[-1]))
    return bytes(group_bits(iter(bits)))
