"""CPU restatement of the reference arithmetic coder -- TEST INFRASTRUCTURE ONLY.

This module is the *checker*: only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it.  The product path
(``lac_amd``) never routes through it.

It restates, in plain Python big-int arithmetic, the algorithm of
``/root/reference/arith_code.py`` (encoder ``A_to_bin``, decoder
``A_from_bin``, predictor ``CDFPredictor``) and of the encode half of
``/root/reference/arithmetic_coding.py`` (``ACSampler``/``Region``/
``CarryBuffer``).  Each function cites the reference lines it follows.  It is
pinned against vectors produced by running the reference itself
(``tools/gen_golden.py`` -> ``tests/golden/``), see tests/test_oracle_golden.py.

Parity is defined on EXACT integer semantics (SURVEY.md finding 3): every table
entry is a Python int, never a wrapping numpy int64.

Tables are given as pmf rows (non-negative ints).  ``rows`` is a sequence of
rows; step i uses ``rows[min(i, len(rows)-1)]`` (a single row = static model).
"""
from __future__ import annotations

import bisect
import itertools


# ---------------------------------------------------------------- predictor
def region_overlap(a, b, c, d):
    """[a,b] with [c,d], closed intervals -- arith_code.py:59-61."""
    return max(0, min(d, b) - max(a, c) + 1)


def cdf_of(pmf):
    """Inclusive running sum (ProbPredictor.calc_dist, arith_code.py:117-123)."""
    return list(itertools.accumulate(int(p) for p in pmf))


def positive_min(cdf):
    """CDFPredictor.minp: smallest positive pmf entry (arith_code.py:79, 81-82)."""
    pdf = itertools.chain([cdf[0]], (cdf[i + 1] - cdf[i] for i in range(len(cdf) - 1)))
    return min(filter(lambda v: v > 0, pdf))


def fudged_dist(cdf, minp, denom):
    """CDFPredictor.fudged_dist, literal loop -- arith_code.py:83-93."""
    if cdf[-1] <= denom * minp:
        return cdf
    res = []
    p = 0
    n = len(cdf)
    for i in range(n):
        d = (cdf[i] * denom) // cdf[-1] - p
        d = max(1, min(denom - p - n + i + 1, d))
        p += d
        res.append(p)
    return res


def symbol_to_range(cdf, minp, s, denom):
    """CDFPredictor.symbol_to_range -- arith_code.py:98-110 (ceil mapping)."""
    return _range_on(fudged_dist(cdf, minp, denom), s, denom)


def _range_on(dist, s, denom):
    """symbol_to_range's arithmetic on an already fudged dist (arith_code.py:102-110)."""
    if s >= len(dist) or s < 0:
        raise AssertionError("unknown symbol", s)
    hd = dist[s]
    ld = dist[s - 1] if s > 0 else 0
    d = dist[-1]
    return (-(-(ld * denom) // d), -(-(hd * denom) // d))


def val_to_symbol(cdf, minp, v, denom):
    """CDFPredictor.val_to_symbol -- arith_code.py:94-97 (bisect_right)."""
    return _symbol_on(fudged_dist(cdf, minp, denom), v, denom)


def _symbol_on(dist, v, denom):
    return bisect.bisect_right(dist, (v * dist[-1]) // denom)


class _Rows:
    """Replay of per-step rows (the 'Replay predictor' of SURVEY.md App. B.2)."""

    def __init__(self, rows):
        self.rows = list(rows)
        self._cache = {}

    def get(self, i):
        i = min(i, len(self.rows) - 1)
        if i not in self._cache:
            cdf = cdf_of(self.rows[i])
            self._cache = {i: (cdf, positive_min(cdf))}
        return self._cache[i]


# ------------------------------------------------------------------ encoder
def encode_digits(rows, symbols, prec, stop=True, trace=None):
    """A_to_bin.run(symbols, stop) -> raw carry digits (arith_code.py:156-211).

    receive_symbol :169-175, decide_bit/emit_bit :176-186, flush :193-202.
    ``trace`` (a list) receives, per symbol, the digits it emitted.
    """
    R = _Rows(rows)
    denom, decision = 1 << prec, 1 << (prec - 1)
    l, h = 0, denom - 1
    out = []
    for i, s in enumerate(symbols):
        cdf, minp = R.get(i)
        w = h - l + 1
        lo, hi = symbol_to_range(cdf, minp, s, w)
        h = l + hi - 1
        l += lo
        step = []
        while (h - l) < decision:
            b = l // decision
            l = l * 2 - b * denom
            h = h * 2 + 1 - b * denom
            step.append(b)
        out.extend(step)
        if trace is not None:
            trace.append(step)
    if stop:
        while l > 0 or h + 1 < denom:
            b = l // decision
            if region_overlap(l, h, b * decision, (b + 1) * decision) < \
               region_overlap(l, h, (b + 1) * decision, (b + 2) * decision):
                b += 1
            l = l * 2 - b * denom
            h = h * 2 + 1 - b * denom
            out.append(b)
    return out


def digits_to_int(digits):
    """A_to_bin.encode: R = sum d_k 2^(L-1-k), returns (R, L) -- arith_code.py:212-219."""
    r = 0
    for v in digits:
        r = (r << 1) + v
    return r, len(digits)


def int_to_bits(R, L):
    return [(R >> (L - 1 - k)) & 1 for k in range(L)]


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


def encode_bytes(rows, symbols, prec):
    """bytes(group_bits(bits(symbols))) as measure_compress does (arith_code.py:420)."""
    R, L = digits_to_int(encode_digits(rows, symbols, prec))
    return bytes(group_bits(int_to_bits(R, L))), L


# ------------------------------------------------------------------ decoders
def decode_bitserial(rows, bits, prec, counts=None):
    """A_from_bin.run(bits, stop=0) restated -- arith_code.py:248-299.

    Returns every symbol the reference decoder determines from ``bits``; with a
    list ``counts``, appends how many symbols each bit's step(bit) yields (:291-298).
    """
    R = _Rows(rows)
    denom, decision = 1 << prec, 1 << (prec - 1)
    l, h, lb, hb = 0, denom - 1, 0, denom - 1
    out = []
    for bit in bits:
        before = len(out)
        wb = (hb - lb + 1) // 2                      # receive_bit :264-267
        lb += wb * bit
        hb = lb + wb - 1
        while True:                                  # decide_symbol :268-273
            cdf, minp = R.get(len(out))
            w = h - l + 1
            ls = val_to_symbol(cdf, minp, lb - l, w)
            hs = val_to_symbol(cdf, minp, hb - l, w)
            if ls != hs:
                break
            lo, hi = symbol_to_range(cdf, minp, ls, w)   # emit_symbol :274-283
            if region_overlap(l + lo, l + hi - 1, lb, hb) == 0:
                raise AssertionError("predictor range does not correspond to val")
            h = l + hi - 1
            l += lo
            out.append(ls)
            while h - l < decision:                  # emit_bit :284-291
                d = l // decision
                l = l * 2 - d * denom
                h = h * 2 + 1 - d * denom
                lb = lb * 2 - d * denom
                hb = hb * 2 + 1 - d * denom
        if counts is not None:
            counts.append(len(out) - before)
    return out


class _Uniform:
    """Predictor(n): floor mapping, no table (arith_code.py:64-74)."""

    def __init__(self, n):
        self.n = n

    def val_to_symbol(self, v, denom):
        return (v * self.n) // denom

    def symbol_to_range(self, s, denom):
        return (s * denom) // self.n, ((s + 1) * denom) // self.n


class _Table:
    """CDFPredictor over replayed rows: step i uses rows[min(i, len-1)].  The
    fudged dist of the current (row, width) is kept: fudged_dist depends on
    nothing else, and the flush ranks every straddled candidate at one width
    (the reference recomputes it per candidate: O(V^2) per flush step at
    V = 32000, tools/gen_golden_flush_long.py)."""

    def __init__(self, rows):
        self.R = _Rows(rows)
        self.i = 0
        self._fd = (None, None, None)

    def _dist(self, denom):
        i = min(self.i, len(self.R.rows) - 1)
        if self._fd[:2] != (i, denom):
            cdf, minp = self.R.get(self.i)
            self._fd = (i, denom, fudged_dist(cdf, minp, denom))
        return self._fd[2]

    def val_to_symbol(self, v, denom):
        return _symbol_on(self._dist(denom), v, denom)

    def symbol_to_range(self, s, denom):
        return _range_on(self._dist(denom), s, denom)


def decode_run(rows, bits, prec, stop=1, uniform=None):
    """A_from_bin.run(bits, stop) restated as a generator -- arith_code.py:248-326:
    the bit-serial decoder of :264-299, then (stop) flush (:300-317), which picks
    among the symbols the window [lb, hb] straddles the one of largest overlap
    ratio (a Python float, ties to the first) and emits it without renormalising,
    until [l, h] lies inside [lb, hb].  Exceptions and partial output are the
    reference's: AssertionError('unknown symbol', V), ZeroDivisionError for a
    zero-width candidate, AssertionError from emit_symbol's overlap check.
    ``uniform=n`` decodes with Predictor(n) instead of the table rows."""
    P = _Uniform(uniform) if uniform else _Table(rows)
    denom, decision = 1 << prec, 1 << (prec - 1)
    st = {"l": 0, "h": denom - 1, "lb": 0, "hb": denom - 1}

    def emit_symbol(s):                               # :274-283
        r = P.symbol_to_range(s, st["h"] - st["l"] + 1)
        if region_overlap(st["l"] + r[0], st["l"] + r[1] - 1, st["lb"], st["hb"]) == 0:
            raise AssertionError("predictor range does not correspond to val")
        st["h"] = st["l"] + r[1] - 1
        st["l"] += r[0]
        if not uniform:
            P.i += 1
        return s

    for bit in bits:
        wb = (st["hb"] - st["lb"] + 1) // 2           # receive_bit :264-267
        st["lb"] += wb * bit
        st["hb"] = st["lb"] + wb - 1
        while True:
            w = st["h"] - st["l"] + 1                 # decide_symbol :268-273
            ls = P.val_to_symbol(st["lb"] - st["l"], w)
            hs = P.val_to_symbol(st["hb"] - st["l"], w)
            if ls != hs:
                break
            s = emit_symbol(ls)
            while st["h"] - st["l"] < decision:       # emit_bit :284-291
                d = st["l"] // decision
                st["l"] = st["l"] * 2 - d * denom
                st["h"] = st["h"] * 2 + 1 - d * denom
                st["lb"] = st["lb"] * 2 - d * denom
                st["hb"] = st["hb"] * 2 + 1 - d * denom
            yield s
    if not stop:
        return

    def k(s):                                         # :305-307
        r = P.symbol_to_range(s, st["h"] - st["l"] + 1)
        return region_overlap(st["lb"] - st["l"], st["hb"] - st["l"], r[0], r[1] - 1) / (r[1] - r[0])

    still = 0
    while not (st["lb"] <= st["l"] and st["h"] <= st["hb"]):   # :308-313
        w = st["h"] - st["l"] + 1
        ls = P.val_to_symbol(st["lb"] - st["l"], w)
        hs = P.val_to_symbol(st["hb"] - st["l"], w)
        before = (st["l"], st["h"])
        yield emit_symbol(max(range(ls, hs + 1), key=k))
        still = still + 1 if (st["l"], st["h"]) == before else 0
        if still >= FLUSH_STILL_LIMIT:                # a full-range symbol: the reference loops forever
            raise RuntimeError("flush does not terminate")
    st.update(l=0, h=denom - 1, lb=0, hb=denom - 1)


FLUSH_STILL_LIMIT = 1000


def decode_value(rows, data_bits, nsym, prec):
    """Value-register decoder, n symbols out.

    Equivalent to ``A_from_bin.run(bits, stop=0)[:n]`` for a valid stream; reads
    zero bits past the end of ``data_bits``.
    """
    R = _Rows(rows)
    P = prec
    denom, decision = 1 << P, 1 << (P - 1)
    nb = len(data_bits)

    def bit(i):
        return data_bits[i] if i < nb else 0

    x = 0
    for i in range(P):
        x = (x << 1) | bit(i)
    pos = P
    l, h = 0, denom - 1
    out = []
    for i in range(nsym):
        cdf, minp = R.get(i)
        w = h - l + 1
        s = val_to_symbol(cdf, minp, x - l, w)
        lo, hi = symbol_to_range(cdf, minp, s, w)
        if not (l + lo <= x <= l + hi - 1):
            raise AssertionError("predictor range does not correspond to val")
        h = l + hi - 1
        l += lo
        out.append(s)
        while h - l < decision:
            d = l // decision
            l = l * 2 - d * denom
            h = h * 2 + 1 - d * denom
            x = x * 2 + bit(pos) - d * denom
            pos += 1
    return out


# --------------------------------------------- arithmetic_coding.py (encode)
def acsampler_cdf(pdf, prec=48):
    """The uint64 CDF ACSampler.sample builds from a float pdf (arithmetic_coding.py:57-72).

    Same numpy float64 operations in the same order: builtin-sum lop bias,
    np.sum normalisation to 2^prec, float cumsum, astype(uint64).
    """
    import numpy as np
    one = 1 << prec
    p = np.array(pdf, dtype=np.float64)
    p += sum(p) / (one / 2 - len(p))
    p *= one / np.sum(p)
    return np.cumsum(p).astype(np.uint64)


def acsampler_encode(cdf, tokens, prec=48):
    """ACSampler encode path on a fixed integer CDF -> output bits.

    Restates sample_scaled_cdf's encode branch (arithmetic_coding.py:78-95),
    Region.map/step/emit/definite (:160-177), CarryBuffer.add/flush (:198-208)
    and flush_compress (:50-56).  ``cdf`` is the uint64 running sum the
    sampler builds (:58-61); on token exhaustion the sampler calls the done
    callback (flush) and then encodes a phantom token 0 whose output is
    detached (:79-84) -- that phantom is not emitted here.
    """
    one = 1 << prec
    low, high = 0, one - 1
    buf, nbuf = 0, 0
    out = []

    def emit():
        nonlocal low, high
        while (high - low + 1) * 2 <= one:
            bit = low >> (prec - 1)
            low = (low << 1) - (bit << prec)
            high = ((high << 1) + 1) - (bit << prec)
            yield bit

    def step(lo_, hi_, d):
        nonlocal low, high
        span = high - low + 1
        low, high = low + (span * lo_) // d, low + (span * hi_) // d - 1
        yield from emit()

    def add(bit):
        nonlocal buf, nbuf
        buf = (buf << 1) + bit
        nbuf += 1
        if high < one:                               # Region.definite :175-177
            yield from flush()

    def flush():
        nonlocal buf, nbuf
        while nbuf > 0:
            nbuf -= 1
            b = buf >> nbuf
            yield b
            buf &= (1 << nbuf) - 1

    denom = int(cdf[-1])
    for tok in tokens:
        lo_ = int(cdf[tok - 1]) if tok else 0
        for bit in step(lo_, int(cdf[tok]), denom):
            out.extend(add(bit))
    for bit in step(1, 2, 3):                        # flush_compress :50-56
        out.extend(add(bit))
    out.extend(flush())
    return out


# ------------------------------------------------ q1 logits quantiser (this repo's format)
def _fmaf(x, k, c):
    """Correctly rounded float32 fma(x, k, c) for float32 arrays (k a power of
    two): the float64 sum is used when it is exact (TwoSum check), otherwise the
    exact rational value is rounded with Fraction."""
    import numpy as np
    from fractions import Fraction
    x = np.asarray(x, dtype=np.float32)
    kx = x.astype(np.float64) * float(k)                               # exact
    cc = np.broadcast_to(np.asarray(c, dtype=np.float32).astype(np.float64), kx.shape)
    with np.errstate(invalid="ignore", over="ignore"):
        s = kx + cc
        exact = ((s - kx) == cc) & ((s - cc) == kx)
        out = s.astype(np.float32)
    for idx in zip(*np.nonzero(~exact & np.isfinite(kx) & np.isfinite(cc))):
        v = Fraction(float(kx[idx])) + Fraction(float(cc[idx]))
        f = np.float32(float(v))                                       # nearest double, then nearest float
        if not np.isfinite(f):                                         # overflow: IEEE rounds to inf
            out[idx] = f
            continue
        lo, hi = np.nextafter(f, np.float32(-np.inf)), np.nextafter(f, np.float32(np.inf))
        cands = [t for t in (lo, f, hi) if np.isfinite(t)]
        best = min((abs(Fraction(float(t)) - v), int(np.float32(t).view(np.uint32)) & 1, t) for t in cands)
        out[idx] = best[2]
    return out


def q1_quantize(logits_f32, prec, tab):
    """Independent numpy restatement of the q1 quantiser for rows
    of float32 logits (bf16 inputs: widen the bit pattern << 16 first)."""
    import numpy as np
    x = np.asarray(logits_f32, dtype=np.float32)
    V = x.shape[-1]
    k = min(24, prec - 1 - (V - 1).bit_length())
    L = 17 * 32
    m = np.fmax.reduce(x, axis=-1, keepdims=True).astype(np.float32)
    with np.errstate(invalid="ignore", over="ignore"):
        c = (np.float32(L) - np.float32(32.0) * m).astype(np.float32)
        y = _fmaf(x, 32.0, c)
        pos = y > 0                                                    # False for NaN
        j = np.where(pos, np.minimum(np.where(pos, y, 0), np.float32(L)), 0).astype(np.int64)
    q = np.asarray(tab, dtype=np.uint64)[L - j] >> np.uint64(24 - k)
    return np.maximum(q, 1).astype(np.uint32)
