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
working.  For them the coders never call ``symbol_to_range``/``val_to_symbol``:
they hand each step's integer pmf row (from ``predictor.dist``) to liblac.so,
whose kernels implement exactly that arithmetic on the device.  A predictor
whose mapping is its own code (``mapping_of`` == 'mapped': overridden
``symbol_to_range`` / ``val_to_symbol`` / ``fudged_dist``, e.g. the reference's
ModifiedMarkov) has no table to scan; ``AC`` gives it the coders of
lac_amd.mapped, which call its methods where the reference does and do the
register arithmetic in liblac's host functions.

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
from .mapped import MappedDecoderMixin, MappedEncoderMixin


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
def _cdf_array(d):
    """An integer CDF as a 1-D int64/uint64 numpy array, or None when it needs exact
    Python ints (object or float arrays, values beyond 64 bits).  Lists go
    through np.fromiter -- never np.asarray, which turns [1, 2**63] into float64."""
    if isinstance(d, np.ndarray):
        return d if d.ndim == 1 and d.dtype.kind in "iu" else None
    for dt in (np.int64, np.uint64):
        try:
            return np.fromiter(d, dtype=dt, count=len(d))
        except (OverflowError, TypeError, ValueError):
            continue
    return None


def _row_of(predictor):
    """(pmf, T): the predictor's current integer pmf row (numpy uint64) from its
    CDF, and the row total as a Python int.  Integer CDFs convert in one
    vectorised pass; anything else through exact Python ints."""
    fast = getattr(predictor, "pmf_row", None)
    if fast is not None:
        r = np.asarray(fast(), dtype=np.uint64)
        return r, int(r.sum(dtype=object)) if r.size else 0
    d = getattr(predictor, "dist", None)
    if d is None:
        raise TypeError(f"{type(predictor).__name__} exposes no probability table (.dist); the GPU coder "
                        "needs CDFPredictor/ProbPredictor-style predictors")
    a = _cdf_array(d)
    if a is not None and a.size:
        if a.dtype.kind == "i" and bool((a < 0).any()):     # before the uint64 cast, which would wrap
            raise ValueError("dist is not monotone non-decreasing")
        a = a.astype(np.uint64, copy=False)
        if a.size > 1 and bool((a[1:] < a[:-1]).any()):
            raise ValueError("dist is not monotone non-decreasing")
        pmf = np.empty(a.size, dtype=np.uint64)
        pmf[0] = a[0]
        np.subtract(a[1:], a[:-1], out=pmf[1:])
        return pmf, int(a[-1])
    cdf = np.asarray([int(x) for x in d], dtype=object)
    pmf = np.empty(len(cdf), dtype=object)
    if len(cdf):
        pmf[0] = int(cdf[0])
        pmf[1:] = cdf[1:] - cdf[:-1]
    if any(int(x) < 0 for x in pmf):
        raise ValueError("dist is not monotone non-decreasing")
    return np.array([int(x) for x in pmf], dtype=np.uint64), int(cdf[-1]) if len(cdf) else 0


_REF_MODULES = ("lac_amd.coder", "arith_code")          # this module and the reference's own


def _impl(predictor, name):
    """(qualname, module) of the function ``type(predictor).<name>`` resolves to."""
    f = getattr(type(predictor), name, None)
    return getattr(f, "__qualname__", None), getattr(f, "__module__", None)


def _is_uniform(predictor):
    """A table-less Predictor(n) with the base class's floor mapping (arith_code.py:64-74)."""
    if getattr(predictor, "dist", None) is not None or not hasattr(predictor, "n"):
        return False
    return all(_impl(predictor, m) in ((f"Predictor.{m}", mod) for mod in _REF_MODULES)
               for m in ("symbol_to_range", "val_to_symbol"))


def _is_table(predictor):
    """A predictor whose mapping is CDFPredictor's over its ``dist`` (arith_code.py:83-110):
    symbol_to_range, val_to_symbol and fudged_dist not overridden.  The reference's
    Llama_AC (llama_compress.py:46-61) restates the first two on numpy arrays; on
    exact integers -- the parity contract, SURVEY.md finding 3 -- they are
    CDFPredictor's, so it counts as a table predictor too."""
    for m in ("symbol_to_range", "val_to_symbol", "fudged_dist"):
        q, mod = _impl(predictor, m)
        if (q, mod) in ((f"CDFPredictor.{m}", x) for x in _REF_MODULES):
            continue
        if q == f"Llama_AC.{m}" and mod in ("llama_compress", "lac_amd.llm"):
            continue
        return False
    return True


def mapping_of(predictor):
    """How AC codes this predictor: 'uniform' (Predictor(n): the floor mapping on the
    GPU), 'table' (CDF tables: the GPU kernels) or 'mapped' (its own
    symbol_to_range / val_to_symbol, evaluated in Python around liblac's host
    register arithmetic, lac_amd.mapped)."""
    if _is_uniform(predictor):
        return "uniform"
    if _is_table(predictor):
        return "table"
    if callable(getattr(predictor, "symbol_to_range", None)) and callable(getattr(predictor, "val_to_symbol", None)):
        return "mapped"
    raise TypeError(f"{type(predictor).__name__} is not a predictor: it needs symbol_to_range and val_to_symbol "
                    "(arith_code.py:64-74) or a CDF table (.dist)")


def _raise_for(code, sym=None):
    if code == _lib.LAC_E_SYMBOL_RANGE:
        raise AssertionError("unknown symbol", sym)
    if code == _lib.LAC_E_DECODE_RANGE:
        raise AssertionError("predictor range does not correspond to val")
    if code == _lib.LAC_E_ZERO_WIDTH:
        raise AssertionError("zero-probability symbol (the reference coder loops forever here)", sym)
    raise _lib.LacError(code, "coder error")


def _is_static(predictor):
    """A table predictor whose accept is the base no-op (Predictor.accept,
    arith_code.py:71-72): its table never changes while it codes -- a static
    model, coded with one stride-0 row (the reference's CDFPredictor fast case,
    fudged_dist returning self.dist, :84-85)."""
    return _impl(predictor, "accept") in (("Predictor.accept", mod) for mod in _REF_MODULES)


def _declared_minp(predictor):
    """The minp the reference's fudge test reads (arith_code.py:84), or None when
    it is by definition the table's smallest positive entry: the base
    ProbPredictor property (:129-131), an O(V) Python scan, is never called."""
    prop = getattr(type(predictor), "minp", None)
    if isinstance(prop, property):
        f = prop.fget
        if getattr(f, "__qualname__", None) == "ProbPredictor.minp" and getattr(f, "__module__", None) in _REF_MODULES:
            return None
    return getattr(predictor, "minp", None)


def fudge_decisions_agree(T, minp, min_pos, prec):
    """Whether fudged_dist's test ``T > w*minp`` (arith_code.py:84) with the
    predictor's ``minp`` and with the table's smallest positive entry
    ``min_pos`` (what the kernels use) agree for every width the coder can
    pass, w in (2^(prec-1), 2^prec].  They differ exactly for the w with
    w*lo < T <= w*hi (lo, hi the two minima in order): refuse only when that
    range meets the coder's.  A minp of 0 (the reference's Llama_AC on rows with
    zero CDF steps, llama_compress.py:43-45) always fudges, and so do the
    kernels when T > 2^prec * min_pos."""
    minp, min_pos = int(minp), int(min_pos)
    if minp == min_pos:
        return True
    lo, hi = min(minp, min_pos), max(minp, min_pos)
    wmin, wmax = (1 << (prec - 1)) + 1, 1 << prec
    first = max(wmin, -(-T // hi))                     # smallest w with T <= w*hi
    last = wmax if lo <= 0 else min(wmax, -(-T // lo) - 1)   # largest w with w*lo < T
    return first > last


class _Tables:
    """Per-step rows from a predictor, converted once per table: a row is cached
    until the coder calls ``accept`` (through :meth:`accept`); a static model
    (``_is_static``) keeps its row -- and its device copy -- for as long as its
    ``dist`` object and ``minp`` stay the same.  A uniform Predictor(n) becomes
    a row of n ones coded with the floor mapping (Predictor.symbol_to_range,
    :69-70)."""

    def __init__(self, predictor, prec=None):
        self.p = predictor
        self.prec = prec
        self.uniform = _is_uniform(predictor)
        self.mapping = "floor" if self.uniform else "ceil"
        self.static = self.uniform or _is_static(predictor)
        self._row = None
        self._key = None
        self._dev = None

    def _static_key(self):
        if self.uniform:
            return (int(self.p.n),)
        return (self.p.dist, getattr(self.p, "minp", None))

    def begin(self):
        """Start of a coder call: rows of adaptive predictors are re-read (the
        caller may have driven the predictor in between)."""
        if not self.static:
            self._row = None

    def row(self):
        if self._row is not None:
            if not self.static:
                return self._row
            k = self._static_key()
            if k[0] is self._key[0] and k[1:] == self._key[1:]:
                return self._row
        self._row = self._build()
        self._dev = None
        if self.static:
            self._key = self._static_key()
        return self._row

    def _build(self):
        if self.uniform:
            return np.ones(int(self.p.n), dtype=np.uint64)
        r, T = _row_of(self.p)
        # fudged_dist decides with the predictor's own minp (arith_code.py:84); the
        # kernels with the row's smallest positive entry (:79-82): a predictor whose
        # minp could change that decision at some width (a stale attribute) is
        # refused instead of being coded with another table
        m = _declared_minp(self.p)
        if m is not None and r.size:
            pos = r[r > 0]
            if pos.size and int(m) != int(pos.min()) and (
                    self.prec is None or not fudge_decisions_agree(T, m, int(pos.min()), self.prec)):
                raise ValueError(f"{type(self.p).__name__}.minp = {int(m)} but its table's smallest positive "
                                 f"entry is {int(pos.min())}, which changes fudged_dist's decision at some "
                                 f"width: the GPU coder derives minp from the table")
        return r

    def row_dev(self, device):
        """The current row on ``device`` (int64 view of the uint64 entries, 1-D)."""
        import torch
        r = self.row()
        if self._dev is None or self._dev.device != device:
            self._dev = torch.from_numpy(r.view(np.int64)).to(device)
        return self._dev

    def accept(self, symbol):
        self.p.accept(symbol)
        if not self.static:
            self._row = None


# ------------------------------------------------------------------ encoder
class A_to_bin:
    """Encoder (arith_code.py:156-246) backed by liblac.so (one stream).  A
    predictor with its own mapping (mapping_of == 'mapped') gets the
    lac_amd.mapped encoder instead.

    A static model (a CDFPredictor whose accept is the base no-op) is coded as
    one stride-0 row: ``run`` / ``encode`` / ``bits`` are one launch over the
    whole symbol sequence, and ``encode`` / ``bits`` of a fresh coder take the
    packed output straight from the device (no per-symbol digit trace).
    Adaptive predictors are streamed in chunks of rows (``_CHUNK_BYTES``)."""

    _CHUNK_BYTES = 32 << 20

    def __new__(cls, predictor=ternary, prec=16):
        if cls is A_to_bin and mapping_of(predictor) == "mapped":
            return object.__new__(_MappedA_to_bin)
        return object.__new__(cls)

    def __init__(self, predictor=ternary, prec=16):
        self.predictor = predictor
        self.precision = prec
        self.denom = 1 << prec
        self.decision = 1 << (prec - 1)
        self.emitted_bits = 0
        self.debug_log = None
        self._coder = None
        self._V = None
        self._tab = None
        self._plane_bits = 0          # output bits held in the device planes since the last reset
        self._nsym = 0                # symbols coded since the last reset

    def _tables(self, begin=True):
        t = self._tab
        if t is None or t.p is not self.predictor:
            t = self._tab = _Tables(self.predictor, self.precision)
        if begin:
            t.begin()
        return t

    # -- device plumbing
    # Digits reach the caller through the per-symbol trace, so the device's own
    # output planes only have to hold what was coded since the last reset (or
    # rebase, which keeps the registers and drops finished words): a stream of
    # any length -- step() loops, repeated run() calls, reuse after flush() --
    # fits a fixed capacity.
    _SLACK = 256                      # flush digits + the word a rebase keeps

    def _fresh(self):
        """Registers at l = 0, h = 2^prec - 1 with nothing coded since (a symbol of
        p > 1/2 narrows l, h without emitting a digit, so empty planes alone do
        not mean fresh registers)."""
        return self._coder is None or (self._plane_bits == 0 and self._nsym == 0)

    def _ensure(self, V, steps):
        per = self.precision + 1      # one symbol emits at most prec digits (renorm)
        need = (steps + 2) * per + self._SLACK
        if self._coder is not None and self._V == V and self._fresh() and self._coder.capacity_bits < need:
            self._coder.close()       # fresh: reallocate at the new size
            self._coder = None
        if self._coder is not None and self._V == V:
            return
        if self._coder is not None and not self._fresh():
            raise RuntimeError(f"table size changed mid-stream ({self._V} -> {V} symbols); flush() first")
        if self._coder is not None:
            self._coder.close()
        self._coder = BatchCoder(V, 1, prec=self.precision, pmf_bits=64, capacity_bits=max(need * 2, 1 << 12))
        self._coder.set_mapping(self._tables(begin=False).mapping)
        self._V = V
        self._plane_bits = 0
        self._nsym = 0

    def _encode_rows(self, rows, syms):
        """Encode syms with ``rows`` -- a [steps, V] array, or one 1-D row for every
        step (a static model, stride 0) -- chunked to the coder's capacity;
        -> (digit lists, (rc, n_ok))."""
        steps = len(syms)
        V = rows.shape[-1]
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
            digs, rc, n_ok = self._encode_chunk(rows if rows.ndim == 1 else rows[i:i + n], syms[i:i + n])
            out.extend(digs)
            if rc:
                return out, (rc, i + n_ok)
            i += n
        return out, (0, steps)

    def _sym_tensor(self, syms):
        """int32 [steps, 1] device symbols; values outside int32 become -1 (the
        kernels report LAC_E_SYMBOL_RANGE for them as for any symbol >= V)."""
        import torch
        if isinstance(syms, np.ndarray):
            a = np.where((syms >= 0) & (syms < 2 ** 31), syms, -1).astype(np.int32)
        else:
            a = np.fromiter((int(s) if 0 <= int(s) < 2 ** 31 else -1 for s in syms), dtype=np.int32,
                            count=len(syms))
        return torch.from_numpy(a).view(len(syms), 1).to(self._coder.device)

    def _encode_chunk(self, rows, syms):
        import torch
        steps = len(syms)
        dev = self._coder.device
        if rows.ndim == 1:
            pmf = self._tab.row_dev(dev)                          # stride 0: one row for every step
        else:
            pmf = torch.from_numpy(np.ascontiguousarray(rows).view(np.int64).reshape(steps, 1, -1)).to(dev)
        tr = torch.zeros((steps, 1, 2), dtype=torch.int64, device=dev)
        self._coder.encode(pmf, self._sym_tensor(syms), trace=tr)
        rc, err, step = self._coder.status()
        t = tr.cpu().numpy()
        # err_step counts symbols since the last reset: the failing one's index in this chunk
        n_ok = steps if rc == 0 else min(max(int(step[0]) - self._nsym, 0), steps)
        self._nsym += n_ok
        digs = [digits_of(int(E), int(k)) for E, k in t[:n_ok, 0]]
        nd = int(t[:n_ok, 0, 1].sum()) if n_ok else 0
        self.emitted_bits += nd
        self._plane_bits += nd
        return digs, rc, n_ok

    # -- registers (reference attributes)
    @property
    def l(self):
        return int(self._coder.registers()[0][0]) if not self._fresh() else 0

    @property
    def h(self):
        return int(self._coder.registers()[1][0]) if not self._fresh() else self.denom - 1

    def __repr__(self):
        sl = bin(self.l + (self.denom << 1))[3:]
        sh = bin(self.h + (self.denom << 1))[3:]
        return f"A_to_bin([{sl[0]}.{sl[1:]},{sh[0]}.{sh[1:]}])"

    # -- reference API
    def step(self, symbol):
        tab = self._tables()
        row = tab.row()
        if self.debug_log:                             # arith_code.py:170 (a truthy list, as there)
            self.debug_log.append((self.l, self.h, "recv", symbol))
        digs, (rc, n_ok) = self._encode_rows(row if tab.static else row[None, :], [symbol])
        if rc:
            _raise_for(rc, symbol)
        if self.debug_log:
            self._log_emits_back(digs[0])
        tab.accept(symbol)
        yield from digs[0]

    def _log_emits_back(self, digits):
        """debug_log's (l, h, 'emit', d) entries (arith_code.py:182) of one symbol: the
        registers before each emit_bit, recovered from the registers after the
        symbol by inverting emit_bit (l = (l' + dD) / 2, h = (h' - 1 + dD) / 2)."""
        l, h = self.l, self.h
        before = []
        for d in reversed(digits):
            l, h = (l + d * self.denom) >> 1, (h - 1 + d * self.denom) >> 1
            before.append((l, h))
        for (l, h), d in zip(reversed(before), digits):
            self.debug_log.append((l, h, "emit", d))

    def __call__(self, symbol):
        if symbol is None:
            return tuple(self.flush())
        return tuple(self.step(symbol))

    def flush(self):
        if self._coder is None:
            self._ensure(len(self._tables().row()), 0)
        l, h = (self.l, self.h) if self.debug_log else (0, 0)
        self._coder.finish()
        rc, err, step = self._coder.status()
        if rc:
            _raise_for(rc)
        fd = self._coder.flush_digits()[0]
        if self.debug_log:
            for d in fd:
                self.debug_log.append((l, h, "emit", d))
                l, h = l * 2 - d * self.denom, h * 2 + 1 - d * self.denom
        self.emitted_bits += len(fd)
        yield from fd
        self._coder.reset()
        self._plane_bits = 0
        self._nsym = 0

    @staticmethod
    def _static_symbols(symbols, V):
        """All symbols as an int64 array, cut after the first one outside [0, V)
        (the reference raises there); -> (array, index of that symbol or None,
        that symbol as given)."""
        syms = symbols if isinstance(symbols, (list, tuple, np.ndarray)) else list(symbols)
        try:
            a = np.asarray(syms, dtype=np.int64).reshape(-1)
        except (OverflowError, TypeError, ValueError):
            a = np.array([int(s) if -2 ** 63 <= int(s) < 2 ** 63 else -1 for s in syms], dtype=np.int64)
        bad = np.flatnonzero((a < 0) | (a >= V))
        if bad.size:
            k = int(bad[0])
            return a[:k + 1], k, syms[k]
        return a, None, None

    def _chunks(self, tab, symbols):
        """(rows, syms, stop_here) batches of an adaptive predictor: at most
        _CHUNK_BYTES of rows each; accept runs for every symbol in range."""
        it = iter(symbols)
        while True:
            rows, syms = [], []
            for s in it:
                r = tab.row()
                rows.append(r)
                syms.append(s)
                if not (0 <= int(s) < len(r)):
                    yield np.stack(rows), syms, True            # the reference raises at this symbol
                    return
                tab.accept(s)
                if len(rows) * r.nbytes >= self._CHUNK_BYTES:
                    break
            if not syms:
                return
            yield np.stack(rows), syms, False

    def run(self, symbols, stop=1):
        if self.debug_log:                             # per-symbol registers for the log
            for sym in symbols:
                yield from self.step(sym)
            if stop:
                yield from self.flush()
            return
        tab = self._tables()
        if tab.static:
            row = tab.row()
            syms, bad, bad_sym = self._static_symbols(symbols, len(row))
            batches = [(row, syms)] if len(syms) else []
        else:
            batches = ((rows, syms) for rows, syms, _ in self._chunks(tab, symbols))
            bad = None
        for rows, syms in batches:
            digs, (rc, n_ok) = self._encode_rows(rows, syms)
            for d in digs:
                yield from d
            if rc:
                _raise_for(rc, bad_sym if bad is not None and n_ok == bad else int(syms[n_ok]))
        if stop:
            yield from self.flush()

    def _encode_static_whole(self, tab, symbols):
        """encode(symbols) of a fresh coder on a static model: one launch, the
        flush and carry resolution on the device, R read from the packed bytes
        (bytes(group_bits(bits())) is exactly R's L-bit binary)."""
        row = tab.row()
        V = len(row)
        syms, bad, bad_sym = self._static_symbols(symbols, V)
        n = len(syms) if bad is None else bad
        self._ensure(V, n)
        if n:
            self._coder.encode(tab.row_dev(self._coder.device), self._sym_tensor(syms[:n]))
            rc, err, step = self._coder.status()
            if rc:
                k = min(max(int(step[0]), 0), n - 1)
                self._nsym = k
                self._plane_bits = 1                   # registers are mid-stream now
                _raise_for(rc, int(syms[k]))
            self._nsym = n
            self._plane_bits = 1
        if bad is not None:
            raise AssertionError("unknown symbol", bad_sym)
        self._coder.finish()
        data, nbits = self._coder.to_bytes()
        L = int(nbits[0])
        R = int.from_bytes(data[0], "big") >> (8 * len(data[0]) - L) if L else 0
        self.emitted_bits += L
        self._coder.reset()
        self._plane_bits = 0
        self._nsym = 0
        return R, L

    def encode(self, symbols, stop=1):
        if stop and not self.debug_log and not isinstance(self, MappedEncoderMixin) and self._fresh():
            tab = self._tables()
            if tab.static:
                return self._encode_static_whole(tab, symbols)
        d = np.fromiter(self.run(symbols, stop), dtype=np.int8)
        return digits_value(d), len(d)

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
        if L:
            b = np.unpackbits(np.frombuffer(r.to_bytes((L + 7) // 8, "big"), dtype=np.uint8))
            yield from b[len(b) - L:].tolist()


def digits_value(d):
    """R = sum d_k 2^(L-1-k) of raw digits d (int8 array: 0..3, and -1 from a
    flush whose l went negative, arith_code.py:193-202) in O(L): each digit
    plane as one binary number, weighted."""
    L = len(d)
    if not L:
        return 0
    pad = (-L) % 8

    def plane(m):
        return int.from_bytes(np.packbits(m.astype(np.uint8)).tobytes(), "big") >> pad

    return plane((d > 0) & (d & 1 == 1)) + (plane(d >= 2) << 1) - plane(d < 0)


# ------------------------------------------------------------------ decoder
_DEC_STATE = np.dtype([("l", "<i8"), ("h", "<i8"), ("x", "<i8"), ("pos", "<u8"), ("nsym", "<i8"),
                       ("err", "<i4"), ("det", "<i4"), ("err_step", "<i8"), ("ndet", "<i8")])   # lac_dec_state
_TAIL_STATE = np.dtype([("l", "<i8"), ("h", "<i8"), ("lb", "<i8"), ("hb", "<i8"), ("err", "<i4"),
                        ("done", "<i4"), ("still", "<i8"), ("nsym", "<i8")])                     # lac_tail_state


def _bit_list(bits):
    """A bit sequence (any iterable of 0 / 1, as the reference's run takes) -> (the bits
    as a sequence of ints -- a list, or a bytearray, which a session appends to and
    indexes alike -- and their bytes packed MSB first: group_bits' format).  Lists and
    tuples of ints go through bytes() and numpy (~0.3 ms per 10^5 bits, against ~25 ms
    for the per-element int() and range checks they take otherwise)."""
    if isinstance(bits, (list, tuple)):
        try:
            raw = bytes(bits)
        except (TypeError, ValueError):
            raw = None
        if raw is not None:
            a = np.frombuffer(raw, dtype=np.uint8)
            if a.size and int(a.max()) > 1:
                raise ValueError("bits are 0 or 1")
            return bytearray(raw), np.packbits(a).tobytes()
    bl = [int(b) for b in bits]
    if any(b not in (0, 1) for b in bl):
        raise ValueError("bits are 0 or 1")
    return bl, np.packbits(np.asarray(bl, dtype=np.uint8)).tobytes()


def _raise_decoder(code, sym=None):
    """The reference's exception for a decoder status (include/lac.h)."""
    if code == _lib.LAC_E_SYMBOL_RANGE:
        raise AssertionError("unknown symbol", sym)                       # arith_code.py:100-101
    if code == _lib.LAC_E_DECODE_RANGE:
        raise AssertionError("predictor range does not correspond to val")   # :277-278
    if code == _lib.LAC_E_FLUSH_ZERO_WIDTH:
        raise ZeroDivisionError("division by zero")                       # flush's k(s), :307
    if code == _lib.LAC_E_FLUSH_LOOP:
        raise RuntimeError("A_from_bin.flush does not terminate here (the reference loops forever, "
                           "arith_code.py:308-313)")
    raise _lib.LacError(code, "decoder error")


class _Session:
    """One bit-serial decoding session of an A_from_bin: the bits received so far
    (host copy, packed MSB first, and its device copy), the predictor's tables,
    and the decoder registers parked on the host between calls -- in the value
    form of the fast decoders (lac_dec_state) while the received window lies
    inside [l, h], in the reference frame (lac_tail_state: l, h, lb, hb) after the
    window has left it or for the flush.  Every symbol decision runs on the GPU."""

    def __init__(self, dec):
        self.dec = dec
        self.prec = dec.precision
        self.tab = _Tables(dec.predictor, dec.precision)
        self.bits = []
        self.buf = np.zeros(64, dtype=np.uint8)
        self.dev = None
        self.nb = None
        self.coder = None
        self.st = np.zeros(1, dtype=_DEC_STATE)          # value form: nothing received yet
        self.st["h"] = dec.denom - 1
        self.st["pos"] = self.prec
        self.st["det"] = 1
        self.st["err_step"] = -1
        self.tst = None                                   # reference frame (tail mode)
        self.stopped_undetermined = False                 # _fast_static stopped before an undetermined symbol
        if self.tab.uniform:
            # Predictor(n)'s val_to_symbol is not the inverse of its floor
            # symbol_to_range, so emit_symbol's overlap check (arith_code.py:277)
            # depends on the window at the bit where a symbol became determined:
            # these streams are decoded bit-serially in the reference frame
            self.tst = np.zeros(1, dtype=_TAIL_STATE)
            self.tst["h"] = dec.denom - 1
            self.tst["hb"] = dec.denom - 1

    # -- plumbing
    def _coder_for(self, V):
        import torch
        if self.coder is None or self.coder.vocab != V:
            if self.coder is not None:
                self.coder.close()
            self.coder = BatchCoder(V, 1, prec=self.prec, pmf_bits=64, capacity_bits=64)
            self.coder.set_mapping(self.tab.mapping)
            self.dev = None
        c = self.coder
        if self.dev is None or self.dev.device != c.device:
            self.dev = torch.from_numpy(self.buf.reshape(1, -1).copy()).to(c.device)
            self.nb = torch.zeros(1, dtype=torch.int64, device=c.device)
        self.nb.fill_(len(self.bits))
        return c

    def _row_dev(self, row, c):
        import torch
        return torch.from_numpy(row.view(np.int64).reshape(1, 1, len(row))).to(c.device)

    def add_bit(self, bit):
        if (len(self.bits) >> 3) + 8 >= len(self.buf):
            self.buf = np.concatenate([self.buf, np.zeros(len(self.buf), dtype=np.uint8)])
            self.dev = None
        n = len(self.bits)
        self.bits.append(bit)
        if bit:
            self.buf[n >> 3] |= 0x80 >> (n & 7)
        if self.dev is not None and (n >> 3) < self.dev.shape[1]:
            self.dev[0, n >> 3] = int(self.buf[n >> 3])      # only the byte the new bit went into
        if self.tst is not None:                             # receive_bit (arith_code.py:264-267)
            t = self.tst
            wb = (int(t["hb"][0]) - int(t["lb"][0]) + 1) // 2
            t["lb"] += wb * bit
            t["hb"] = int(t["lb"][0]) + wb - 1
            return
        st = self.st
        pos = int(st["pos"][0])
        if bit and pos - self.prec <= n < pos:               # was read as a padding 0
            st["x"] += 1 << (pos - 1 - n)

    def load_bits(self, bl, data):
        """Take a whole bit list at once (the fast path): the same buffers add_bit builds."""
        self.bits = bl if isinstance(bl, (list, bytearray)) else list(bl)
        self.buf = np.zeros(max(64, ((len(bl) >> 3) + 8) * 2 + 7 & ~7), dtype=np.uint8)   # rows 8-byte aligned
        self.buf[:len(data)] = np.frombuffer(data, dtype=np.uint8)
        self.dev = None
        x = 0
        for i in range(self.prec):                        # the first window, 0s past the end
            x = (x << 1) | (self.bits[i] if i < len(self.bits) else 0)
        self.st["x"] = x

    # -- decisions
    def decide(self):
        """Every symbol the bits received so far determine (decide_symbol /
        emit_symbol / emit_bit, arith_code.py:268-299), yielded one at a time."""
        while self.tst is None:
            row = self.tab.row()
            c = self._coder_for(len(row))
            c.decode_open(self.dev, self.nb)
            trial = self.st.copy()
            trial["det"] = 1
            trial["ndet"] = 0
            check(c.lib.lac_decode_set_state(c.ctx, trial.ctypes.data_as(C.c_void_p), c._stream))
            s = int(c.decode(self._row_dev(row, c)).cpu()[0, 0])
            new = np.zeros(1, dtype=_DEC_STATE)
            check(c.lib.lac_decode_get_state(c.ctx, new.ctypes.data_as(C.c_void_p), c._stream))
            if int(new["err"][0]):
                # the window has left [l, h] (foreign or corrupt bits): continue in the
                # reference's frame, where the reference raises or (uniform
                # Predictor) emits out-of-range symbols
                self.to_tail()
                break
            if int(new["ndet"][0]) != 1:
                return                                       # not determined by the bits so far
            self.st = new
            self.tab.accept(s)
            yield s
        while True:
            code, s = self.tail_step(_lib.LAC_TAIL_DECIDE)
            if code == 1:
                return
            self.tab.accept(s)
            yield s

    def to_tail(self):
        """Value-form registers -> l, h, lb, hb (lac_decode_tail_begin)."""
        row = self.tab.row()
        c = self._coder_for(len(row))
        c.decode_open(self.dev, self.nb)
        st = self.st.copy()
        check(c.lib.lac_decode_set_state(c.ctx, st.ctypes.data_as(C.c_void_p), c._stream))
        check(c.lib.lac_decode_tail_begin(c.ctx, c._stream))
        self.tst = np.zeros(1, dtype=_TAIL_STATE)
        check(c.lib.lac_decode_tail_get_state(c.ctx, self.tst.ctypes.data_as(C.c_void_p), c._stream))

    def tail_step(self, mode):
        """One DECIDE / FLUSH step on the GPU -> (code, symbol); raises the
        reference's exception on an error."""
        import torch
        row = self.tab.row()
        c = self._coder_for(len(row))
        check(c.lib.lac_decode_tail_set_state(c.ctx, self.tst.ctypes.data_as(C.c_void_p), c._stream))
        pmf = None if self.tab.uniform else self._row_dev(row, c)
        out = torch.zeros(2, dtype=torch.int64, device=c.device)
        check(c.lib.lac_decode_tail_step(c.ctx, C.c_void_p(pmf.data_ptr()) if pmf is not None else None, 0, mode,
                                         C.c_void_p(out.data_ptr()), C.c_void_p(out.data_ptr() + 8), c._stream))
        check(c.lib.lac_decode_tail_get_state(c.ctx, self.tst.ctypes.data_as(C.c_void_p), c._stream))
        sym, code = out.cpu().tolist()
        code = int(np.int64(code).astype(np.int32))           # int32 code in the low half
        if code < 0:
            _raise_decoder(code, sym)
        return code, sym

    def flush(self):
        """A_from_bin.flush (arith_code.py:300-317), one GPU step per symbol."""
        if self.tst is None:
            self.to_tail()
        while True:
            code, s = self.tail_step(_lib.LAC_TAIL_FLUSH)
            if code == 1:
                return
            self.tab.accept(s)
            yield s

    def close(self):
        if self.coder is not None:
            self.coder.close()
            self.coder = None


class A_from_bin:
    """Decoder (arith_code.py:248-334) backed by liblac.so (one stream).

    ``run(bits, stop)``, ``step(bit)`` / ``__call__(bit)``, ``flush()`` /
    ``__call__(None)`` and ``decode(R, L, stop)`` yield exactly the symbols the
    reference yields, in the same order, and raise where it raises (its flush
    included: SURVEY.md finding 5; golden vectors tests/golden/flush_cases.json).
    The stream does not record its symbol count; ``run(bits, n=...)`` is this
    build's extension that decodes exactly n symbols (zero bits past the end).
    """

    def __new__(cls, predictor=ternary, prec=16):
        if cls is A_from_bin and mapping_of(predictor) == "mapped":
            return object.__new__(_MappedA_from_bin)
        return object.__new__(cls)

    def __init__(self, predictor=ternary, prec=16):
        self.predictor = predictor
        self.precision = prec
        self.denom = 1 << prec
        self.decision = 1 << (prec - 1)
        self._sess = None

    def run(self, bits, stop=1, n=None, max_symbols=1 << 24):
        """A_from_bin.run (arith_code.py:322-326), a generator like the reference's.

        A fresh decoder takes the whole bit list at once: the fast value-form
        decoder finds the determined symbols (one GPU decode per symbol), the
        reference-frame tail continues where the window leaves [l, h], and
        ``stop`` runs the flush.  A decoder that already holds a stream (step()
        calls, a run(..., stop=0)) continues it bit by bit, as the reference does.
        With ``n``: exactly n symbols of a fresh stream, no flush (this build's
        extension; ``max_symbols`` bounds the count-free form)."""
        if n is not None:
            bl = [int(b) for b in bits]
            if _is_uniform(self.predictor):
                return iter(self._uniform_n(bl, n))
            return iter(self._decode_bytes(bytes(group_bits(iter(bl))), len(bl), n))
        return self._run(bits, stop, max_symbols)

    def _uniform_n(self, bl, n):
        """n symbols of a Predictor(n) stream: the reference's bit-serial decoder
        over the bits, then zero bits, until n symbols are out."""
        out = []
        sess = _Session(self)
        try:
            i = 0
            while len(out) < n:
                sess.add_bit(bl[i] if i < len(bl) else 0)
                out.extend(sess.decide())
                i += 1
                if i > len(bl) + 4 * (n + 1) * self.precision:
                    raise AssertionError("predictor range does not correspond to val")
        finally:
            sess.close()
        return out[:n]

    def _run(self, bits, stop, max_symbols):
        if self._sess is not None:
            for b in bits:
                yield from self.step(b)
        else:
            bl, data = _bit_list(bits)
            yield from self._fast(bl, max_symbols, data)
        if stop:
            yield from self.flush()

    def _fast(self, bl, max_symbols, data=None):
        """Determined symbols of a whole bit list: value-form decode per symbol;
        the registers before a symbol the bits do not determine (or that fails)
        are restored and parked as this decoder's session."""
        sess = self._sess = _Session(self)
        if sess.tst is not None:                   # Predictor(n): bit-serial (see _Session)
            for b in bl:
                sess.add_bit(b)
                yield from sess.decide()
            return
        if data is None:
            data = np.packbits(np.asarray(bl, dtype=np.uint8)).tobytes()     # group_bits' format
        sess.load_bits(bl, data)
        tab = sess.tab
        if tab.static:
            yield from self._fast_static(sess, max_symbols)
            if not sess.stopped_undetermined:          # (else decide() would find the same)
                yield from sess.decide()
            return
        for _ in range(max_symbols):
            row = tab.row()
            c = sess._coder_for(len(row))
            c.decode_open(sess.dev, sess.nb)
            st = sess.st.copy()
            check(c.lib.lac_decode_set_state(c.ctx, st.ctypes.data_as(C.c_void_p), c._stream))
            s = int(c.decode(sess._row_dev(row, c)).cpu()[0, 0])
            new = np.zeros(1, dtype=_DEC_STATE)
            check(c.lib.lac_decode_get_state(c.ctx, new.ctypes.data_as(C.c_void_p), c._stream))
            if int(new["err"][0]) or int(new["ndet"][0]) != int(st["ndet"][0]) + 1:
                break
            sess.st = new
            tab.accept(s)
            yield s
        yield from sess.decide()                   # undetermined: nothing; window off [l, h]: the reference's way

    def _fast_static(self, sess, max_symbols):
        """Determined symbols of a static model in a few launches: chunks of
        stride-0 steps (doubling) decoded with LAC_OPT_DECODE_STOP, so the stream
        stops by itself before the first symbol the bits do not determine (or whose
        window leaves [l, h]) with the registers of that point: the session parks
        exactly where the per-symbol loop would, and nothing is decoded twice (round
        5 replayed the last chunk up to that point: every symbol decoded twice)."""
        tab = sess.tab
        row = tab.row()
        V = len(row)
        c = sess._coder_for(V)
        c.decode_open(sess.dev, sess.nb)
        start = sess.st.copy()
        start["det"] = 1
        check(c.lib.lac_decode_set_state(c.ctx, start.ctypes.data_as(C.c_void_p), c._stream))
        pmf = tab.row_dev(c.device).view(1, 1, V)
        # first chunk: the bits over the table's entropy (+10 %), what a stream drawn
        # from the table holds; doubling covers the rest, the stop the overshoot
        p = row[row > 0].astype(np.float64)
        p /= p.sum()
        H = float(-(p * np.log2(p)).sum())
        done, n = 0, int(min(1 << 20, 64 + 1.1 * len(sess.bits) / max(H, 1e-9)))
        c.set_decode_stop(True)
        try:
            while done < max_symbols:
                n = min(n, max_symbols - done)
                out = c.decode(pmf.expand(n, 1, V))
                new = np.zeros(1, dtype=_DEC_STATE)
                check(c.lib.lac_decode_get_state(c.ctx, new.ctypes.data_as(C.c_void_p), c._stream))
                err = int(new["err"][0])
                sess.stopped_undetermined = err == _lib.LAC_E_UNDETERMINED
                # the stream stopped (undetermined) or failed at err_step with the registers of
                # that point; every symbol before it is determined
                got = (int(new["err_step"][0]) if err else int(new["nsym"][0])) - int(start["nsym"][0])
                got = max(min(got, n), 0)
                syms = out[:got, 0].cpu().tolist() if got else []
                if err:
                    new["err"] = 0
                    new["err_step"] = -1
                    new["nsym"] = start["nsym"][0] + got
                    new["ndet"] = start["ndet"][0] + got
                    new["det"] = 1
                    check(c.lib.lac_decode_set_state(c.ctx, new.ctypes.data_as(C.c_void_p), c._stream))
                start = new
                sess.st = start
                # a static model's accept is the base no-op (_is_static): the reference calls
                # it per symbol to no effect, so the symbols go out without the calls
                yield from syms
                done += got
                if err or got < n:
                    return
                n *= 2
        finally:
            c.set_decode_stop(False)

    # ---- registers (arith_code.py:249-263): l, h and the received-bit interval [lb, hb]
    def _regs(self):
        d = self.denom
        if self._sess is None:
            return 0, d - 1, 0, d - 1
        if self._sess.tst is not None:
            t = self._sess.tst
            return int(t["l"][0]), int(t["h"][0]), int(t["lb"][0]), int(t["hb"][0])
        st = self._sess.st
        past = int(st["pos"][0]) - len(self._sess.bits)
        pad = min(max(past, 0), self.precision)
        x = int(st["x"][0])
        return int(st["l"][0]), int(st["h"][0]), x, x + (1 << pad) - 1

    @property
    def l(self):
        return self._regs()[0]

    @property
    def h(self):
        return self._regs()[1]

    @property
    def lb(self):
        return self._regs()[2]

    @property
    def hb(self):
        return self._regs()[3]

    def __repr__(self):
        sl = bin(self.l + (self.denom << 1))[3:]
        sh = bin(self.h + (self.denom << 1))[3:]
        slb = bin(self.lb + (self.denom << 1))[3:]
        shb = bin(self.hb + (self.denom << 1))[3:]
        slb = "".join(slb[i] for i in range(len(slb)) if slb[i] == shb[i])
        return f"A_from_bin([{sl[0]}.{sl[1:]},{sh[0]}.{sh[1:]}],{slb[0]}.{slb[1:]})"

    # ---- bit-serial decoding: step(bit) / __call__ (arith_code.py:291-298, 318-321)
    def step(self, bit):
        """receive_bit + the decide_symbol / emit_symbol loop (arith_code.py:291-298):
        yields, once each, the symbols that the bits received so far determine --
        the same symbols after the same bits as the reference, raising where it
        raises.

        The GPU decides; between calls the decoder's registers wait on the host
        (include/lac.h lac_decode_get_state / set_state, lac_decode_tail_*).  In
        the value form each call tries the next symbol against the bits so far,
        zero-padded, and commits it only when the 0- and 1-padded ends of the
        window agree (the reference's ls == hs); a bit inside the value window is
        added to x where it was read as 0.  A window that leaves [l, h] moves the
        session to the reference frame (l, h, lb, hb), where receive_bit is a
        host-side halving and each decision one tail step."""
        bit = int(bit)
        if bit not in (0, 1):
            raise ValueError("bits are 0 or 1")
        if self._sess is None:
            self._sess = _Session(self)
        self._sess.add_bit(bit)
        return self._sess.decide()

    def flush(self):
        """A_from_bin.flush (arith_code.py:300-317): while [l, h] is not inside the
        received window, emit the straddled symbol of largest overlap ratio; then
        the registers reset (the next bits start a new stream)."""
        sess, self._sess = self._sess, None
        if sess is None:
            return                                  # fresh registers: [l, h] == [lb, hb], nothing to emit
        try:
            yield from sess.flush()
        finally:
            sess.close()

    def __call__(self, bit):
        if bit is None:
            return tuple(self.flush())
        return tuple(self.step(bit))

    def decode(self, bits, length, stop=1, n=None):
        """A_from_bin.decode(int, length, stop) -- arith_code.py:327-334 (run over
        the length bits of ``bits``, MSB first; with stop, the flush and a second,
        idle one)."""
        bl = [(bits >> (length - 1 - i)) & 1 for i in range(length)]
        if n is not None:
            return self.run(bl, stop, n)
        return self._decode_gen(bl, stop)

    def _decode_gen(self, bl, stop):
        yield from self._run(bl, stop, 1 << 24)
        if stop:
            yield from self.flush()

    def _decode_bytes(self, data, nbits, n, max_symbols=1 << 24):
        import torch
        tab = _Tables(self.predictor, self.precision)
        out = []
        coder = None
        limit = n if n is not None else max_symbols
        try:
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
                if tab.static and n is not None:         # a static model: all n symbols in one launch
                    syms = coder.decode(tab.row_dev(coder.device).view(1, 1, V).expand(n - i, 1, V))
                    rc, err, step = coder.status()
                    if rc:
                        _raise_for(int(err[0]) or _lib.LAC_E_DECODE_RANGE)
                    for s in syms[:, 0].cpu().tolist():
                        out.append(s)
                        tab.accept(s)
                    break
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
                tab.accept(s)
        finally:
            if coder is not None:
                coder.close()
        return out


class _MappedA_to_bin(MappedEncoderMixin, A_to_bin):
    def __init__(self, predictor=ternary, prec=16):
        self._mapped_init(predictor, prec)


class _MappedA_from_bin(MappedDecoderMixin, A_from_bin):
    def __init__(self, predictor=ternary, prec=16):
        self._mapped_init(predictor, prec)


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
    """bytes(group_bits(comp.bits(inp))) with progress lines -- arith_code.py:401-420.

    The input is consumed lazily, as ``comp.bits`` pulls it, and every output
    bit is appended to ``save_bits``.  A progress line ("n -> entropy  bits/tok",
    carriage-return terminated) is printed as each input arrives while the
    output count is a multiple of ``print_every_inp`` (the reference tests the
    output count there, :409) and after every ``print_every_out`` output bits.
    The coder reads its input in chunks ahead of the bits it yields, so the
    output count stands still while a chunk is read: the input side prints at
    most once per output count (the reference, whose bits interleave with its
    inputs, prints on each input only while the count sits at a multiple)."""
    if save_bits is None:
        save_bits = []
    n_in = n_out = 0
    last = None
    printed_at = None                                   # output count of the last input-side line

    def progress():
        info = comp.total_encoded_entropy
        print(n_in, "->", info, "   ", info / n_in, " bits/tok ", inp_cb(last), end="        \r")

    def inputs():
        nonlocal n_in, last, printed_at
        for v in inp:
            yield v
            last = v
            n_in += 1
            if n_out % print_every_inp == 0 and n_out != printed_at:
                printed_at = n_out
                progress()

    def outputs(bits):
        nonlocal n_out
        for b in bits:
            save_bits.append(b)
            yield b
            n_out += 1
            if n_out % print_every_out == 0:
                progress()

    return bytes(group_bits(outputs(comp.bits(inputs()))))
