"""Host side of the drop-in surface (no GPU): table conversion, static-model
detection, row caching, the digit fold and measure_compress's lazy consumption
(lac_amd/coder.py; the reference's arith_code.py:76-135, 207-219, 401-420)."""
import itertools
import time

import numpy as np
import pytest

from lac_amd.coder import (CDFPredictor, Predictor, ProbPredictor, _row_of, _Tables, digits_value,
                           measure_compress)


def _exact_pmf(cdf):
    c = [int(x) for x in cdf]
    return [c[0]] + [c[i + 1] - c[i] for i in range(len(c) - 1)]


@pytest.mark.parametrize("kind", ["list", "int64", "uint64", "object", "big_list"])
def test_row_of_equals_exact_int_conversion(kind):
    """Vectorised CDF -> pmf conversion == the exact Python-int difference, for
    list / numpy int64 / uint64 / object CDFs and totals past 2^63."""
    rng = np.random.default_rng(3)
    for _ in range(20):
        V = int(rng.integers(1, 2000))
        top = 62 if kind != "big_list" else 63
        pmf = [int(x) for x in rng.integers(0, 1 << (top - 12), V, dtype=np.uint64)]
        if kind == "big_list":
            pmf[0] += 1 << 63                  # the total lands in [2^63, 2^64)
        cdf = list(itertools.accumulate(pmf))
        d = {"list": lambda: cdf, "big_list": lambda: cdf, "int64": lambda: np.asarray(cdf, dtype=np.int64),
             "uint64": lambda: np.asarray(cdf, dtype=np.uint64),
             "object": lambda: np.asarray(cdf, dtype=object)}[kind]()
        p = CDFPredictor.__new__(CDFPredictor)
        p.dist = d
        r, T = _row_of(p)
        assert r.dtype == np.uint64 and [int(x) for x in r] == pmf and T == cdf[-1]


def test_row_of_refuses_decreasing_cdf():
    for d in ([3, 2, 5], np.array([3, 2, 5]), np.array([-1, 2, 5]), np.array([3, 2, 5], dtype=np.uint64)):
        p = CDFPredictor.__new__(CDFPredictor)
        p.dist = d
        with pytest.raises(ValueError):
            _row_of(p)


def test_static_model_detection_and_row_cache():
    """A CDFPredictor (accept = the base no-op) is a static model: one row,
    converted once, re-converted only when its dist object or minp changes;
    ProbPredictor-style predictors re-read their table after every accept."""
    p = CDFPredictor([2, 9, 10])
    t = _Tables(p, 16)
    assert t.static and not t.uniform
    r = t.row()
    assert t.row() is r
    t.accept(1)
    assert t.row() is r                        # accept is a no-op: same table
    p.dist = [5, 8, 40]
    p.minp = 3
    assert list(t.row()) == [5, 3, 32]
    assert _Tables(Predictor(7), 16).static and _Tables(Predictor(7), 16).uniform

    class Count(ProbPredictor):
        def __init__(self):
            super().__init__(3)
            self.k = 1

        def prob(self, s):
            return self.k + s

        def accept(self, s):
            self.k += 1
            super().accept(s)

    q = Count()
    tq = _Tables(q, 16)
    assert not tq.static
    assert list(tq.row()) == [1, 2, 3]
    tq.accept(0)
    assert list(tq.row()) == [2, 3, 4]


def test_probpredictor_base_minp_not_called():
    """The base ProbPredictor.minp (arith_code.py:129-131, an O(V) Python scan) is
    the table's positive minimum by definition: the coder never evaluates it."""
    calls = []

    class P(ProbPredictor):
        def __init__(self):
            super().__init__(5)

        def prob(self, s):
            return s + 1

    orig = ProbPredictor.minp.fget
    try:
        ProbPredictor.minp = property(lambda self: calls.append(1) or orig(self))
        ProbPredictor.minp.fget.__qualname__ = "ProbPredictor.minp"
        ProbPredictor.minp.fget.__module__ = "lac_amd.coder"
        assert list(_Tables(P(), 16).row()) == [1, 2, 3, 4, 5]
        assert not calls
    finally:
        ProbPredictor.minp = property(orig)


def test_numpy_cdf_probpredictor_host_time_per_token():
    """a ProbPredictor returning a numpy int64 CDF at V=32000
    costs the coder <= 1 ms of host time per token (was 24 ms: object-dtype
    conversion + the reference's O(V) minp)."""
    from lac_amd import synth
    cdfs = [np.cumsum(synth.pmf_row(77, t, 0, 32000, "loguniform", 24).astype(np.int64)) for t in range(4)]

    class NP(ProbPredictor):
        def __init__(self):
            super().__init__(32000)
            self.i = 0

        def calc_dist(self):
            self.dcache = cdfs[self.i % 4]
            return self.dcache

        def accept(self, s):
            self.i += 1
            super().accept(s)

    t = _Tables(NP(), 48)
    for _ in range(8):
        t.row()
        t.accept(0)
    t0 = time.perf_counter()
    n = 200
    for _ in range(n):
        r = t.row()
        t.accept(0)
    per = (time.perf_counter() - t0) / n
    assert r.dtype == np.uint64 and per < 1e-3, per


def test_digits_value_is_the_reference_fold():
    """encode()'s R from raw digits (0..3, and -1 from a flush) == the reference's
    r = 2r + d fold (arith_code.py:212-219)."""
    rng = np.random.default_rng(9)
    for _ in range(300):
        n = int(rng.integers(0, 200))
        d = rng.choice([-1, 0, 1, 2, 3], size=n, p=[0.02, 0.45, 0.45, 0.05, 0.03]).astype(np.int8)
        r = 0
        for v in d.tolist():
            r = 2 * r + v
        assert digits_value(d) == r


class _LazyComp:
    """A stand-in coder that pulls one input per output bit (as the reference's
    bits() does through run/step) and records the interleaving."""

    def __init__(self, log):
        self.log = log
        self.total_encoded_entropy = 0.0

    def bits(self, inp):
        for v in inp:
            self.log.append(("in", v))
            self.total_encoded_entropy += 1.5
            yield v & 1


def test_measure_compress_is_lazy_and_prints_progress(capsys):
    """measure_compress consumes its input as the coder pulls it (a generator is
    never listed first) and prints the reference's progress lines
    (arith_code.py:401-420): on inputs while the output count is a multiple of
    print_every_inp, and every print_every_out outputs."""
    log = []

    def gen():
        for i in range(10):
            log.append(("gen", i))
            yield i

    saved = []
    out = measure_compress(_LazyComp(log), gen(), print_every_out=4, print_every_inp=3, save_bits=saved)
    assert log[:4] == [("gen", 0), ("in", 0), ("gen", 1), ("in", 1)]     # interleaved: lazy
    assert saved == [i & 1 for i in range(10)]
    assert out == bytes([0b01010101, 0b01000000])
    lines = capsys.readouterr().out.split("\r")
    # an input is counted when the coder asks for the next one, after i outputs:
    # counts 3, 6, 9 print; outputs 4 and 8 print -- 5 lines, as the reference's
    # measure_compress prints for this coder (checked in the build container)
    assert sum(1 for ln in lines if "bits/tok" in ln) == 5


def test_bit_list_fast_path_equals_generic():
    """A_from_bin.run's bit conversion (coder._bit_list): lists / tuples of ints and bools
    take bytes() + numpy, anything else (numpy ints, floats, strings, generators) the
    per-element int(); both give the same bits and packed bytes, and values other than
    0 / 1 raise ValueError either way."""
    from lac_amd.coder import _bit_list
    rng = np.random.default_rng(4)
    for n in (0, 1, 7, 8, 9, 1000, 100001):
        bits = [int(b) for b in rng.integers(0, 2, n)]
        want = (bits, np.packbits(np.asarray(bits, dtype=np.uint8)).tobytes())
        for form in (bits, tuple(bits), [bool(b) for b in bits], [np.int64(b) for b in bits],
                     [float(b) for b in bits], [str(b) for b in bits], iter(bits)):
            bl, data = _bit_list(form)
            assert list(bl) == want[0] and data == want[1]
            assert all(type(b) is int for b in bl) and isinstance(bl, (list, bytearray))
    for bad in ([0, 1, 2], [0, -1], (1, 256), [0, 1, 2.0], iter([1, 3])):
        with pytest.raises(ValueError):
            _bit_list(bad)
