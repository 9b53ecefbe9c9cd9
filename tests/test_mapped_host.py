"""Predictors with their own mapping against the reference.

tests/golden/custom_cases.json records what the reference coder does with the
predictors of tests/custom_predictors.py (tools/gen_golden_custom.py): encoded
bits, A_to_bin.debug_log, and A_from_bin.run(bits, stop=1 / 0) with its
exception.  AC routes these predictors to lac_amd.mapped (their Python mapping
around liblac's host register functions, no GPU needed), never to the table
kernels; table predictors are refused when their minp disagrees with the table.
"""
import numpy as np
import pytest

import custom_predictors
from conftest import load_golden

DATA = load_golden("custom_cases.json")


def _classes():
    from lac_amd.coder import CDFPredictor, Predictor
    return custom_predictors.make(Predictor, CDFPredictor)


def _drain(gen):
    out = []
    try:
        for v in gen:
            out.append(int(v))
    except Exception as e:                      # noqa: BLE001 -- compared with the recorded one
        return out, [type(e).__name__, str(e.args[0]) if e.args else ""]
    return out, None


def test_dispatch_by_mapping():
    from lac_amd import coder
    from lac_amd.llm import Llama_AC
    from lac_amd.mapped import MappedDecoderMixin, MappedEncoderMixin
    Fixed, FloorCDF, Counting = _classes()
    assert coder.mapping_of(coder.Predictor(3)) == "uniform"
    assert coder.mapping_of(coder.CDFPredictor([1, 3, 4])) == "table"
    assert coder.mapping_of(coder.ProbPredictor(5)) == "table"
    assert coder.mapping_of(Llama_AC.__new__(Llama_AC)) == "table"
    for p in (Fixed([1, 2, 3]), FloorCDF([1, 3, 4]), Counting(4)):
        assert coder.mapping_of(p) == "mapped"
        ac = coder.AC(p, 16)
        assert isinstance(ac.to_bin, coder.A_to_bin) and isinstance(ac.to_bin, MappedEncoderMixin)
        assert isinstance(ac.from_bin, coder.A_from_bin) and isinstance(ac.from_bin, MappedDecoderMixin)
    with pytest.raises(TypeError):
        coder.mapping_of(object())


@pytest.mark.parametrize("i", range(len(DATA["cases"])))
def test_mapped_coder_matches_reference(i):
    from lac_amd.coder import AC
    c = DATA["cases"][i]
    cls = _classes()

    def mk():
        return custom_predictors.build(c["kind"], *cls, c["params"])
    enc = AC(mk(), c["prec"]).to_bin
    enc.debug_log = ["start"]
    if "encode_exc" in c:                       # the reference loops forever on a zero-width range
        assert c["encode_exc"] == "timeout"
        with pytest.raises(AssertionError):
            list(enc.bits(c["syms"]))
        return
    bits = list(enc.bits(c["syms"]))
    assert "".join(map(str, bits)) == c["bits"]
    assert [list(x) if isinstance(x, tuple) else x for x in enc.debug_log] == c["debug_log"]
    for stop in (1, 0):
        want = c[f"stop{stop}"]
        got = _drain(AC(mk(), c["prec"]).from_bin.run(iter(bits), stop=stop))
        assert [got[0], got[1]] == [want[0], want[1]], stop


def test_table_predictor_with_stale_minp_is_refused():
    """CDFPredictor's fudge test uses the predictor's minp (arith_code.py:84); a
    subclass that swaps tables without updating it would be coded with another
    decision by kernels that take minp from the table: refused, not silently coded."""
    from lac_amd.coder import CDFPredictor, _Tables

    class Swap(CDFPredictor):
        def accept(self, s):
            self.dist = [5, 8, 40]               # minp stays the first table's

    p = Swap([2, 9, 10])
    assert list(_Tables(p, 6).row()) == [2, 7, 1]
    p.accept(0)
    # minp 1 against the table's 3: T = 40 fudges for w < 40 with minp 1 and for
    # w < 14 with 3 -- at prec 6 (w in 33..64) the decisions differ at w = 33..39
    with pytest.raises(ValueError):
        _Tables(p, 6).row()
    with pytest.raises(ValueError):
        _Tables(p).row()                         # no precision given: equality required
    # at prec 16 (w > 2^15) neither fudges: the same code either way, accepted
    assert list(_Tables(p, 16).row()) == [5, 3, 32]
    p.minp = 3
    assert list(_Tables(p, 6).row()) == [5, 3, 32]


def test_fudge_decisions_agree_matches_brute_force():
    """fudge_decisions_agree == 'T > w*minp' and 'T > w*min_pos' agree for every w
    in (2^(prec-1), 2^prec] (arith_code.py:84), minp 0 included (Llama_AC on rows
    with zero CDF steps, llama_compress.py:43-45)."""
    import random
    from lac_amd.coder import fudge_decisions_agree
    rng = random.Random(5)
    for _ in range(3000):
        prec = rng.randint(2, 9)
        T = rng.randint(1, 1 << rng.randint(1, 14))
        m1, m2 = rng.randint(0, 300), rng.randint(1, 300)
        ws = range((1 << (prec - 1)) + 1, (1 << prec) + 1)
        want = all((T > w * m1) == (T > w * m2) for w in ws)
        assert fudge_decisions_agree(T, m1, m2, prec) == want, (T, m1, m2, prec)


def test_llama_minp_zero_rows_accepted_when_both_fudge():
    """a Llama_AC row whose float cumsum has zero steps has
    minp 0 -- the reference always fudges.  The kernels fudge when T > 2^prec *
    min_pos; with T ~ 2^60 at prec 48 both always fudge, so the row is coded
    (it was refused); a table where the kernels would not fudge is still refused."""
    from lac_amd.coder import ProbPredictor, _Tables

    class ZeroStep(ProbPredictor):
        def __init__(self, cdf):
            super().__init__(len(cdf))
            self.cdf = cdf

        def calc_dist(self):
            self.dcache = self.cdf
            return self.dcache

        @property
        def minp(self):                           # Llama_AC's: zeros included
            return int(min(self.dist[0], np.min(np.diff(self.dist))))

    cdf = np.cumsum(np.array([2, 0, 5, 1 << 59, 0, 3], dtype=np.int64))
    p = ZeroStep(cdf)
    assert p.minp == 0
    assert list(_Tables(p, 48).row()) == [2, 0, 5, 1 << 59, 0, 3]
    small = ZeroStep(np.cumsum(np.array([4, 0, 4], dtype=np.int64)))
    with pytest.raises(ValueError):
        _Tables(small, 48).row()


def test_mapped_range_beyond_int64_is_refused():
    """ADVICE/VERDICT r3: a predictor whose symbol_to_range returns a bound beyond
    int64 is refused (LacError), not wrapped by ctypes ((1 << 64) + 5 -> 5)."""
    from lac_amd._lib import LacError
    from lac_amd.coder import AC, Predictor

    class Wide(Predictor):
        def symbol_to_range(self, s, denom):
            return (1 << 64) + 5, (1 << 64) + 9

        def val_to_symbol(self, v, denom):
            return 0

    with pytest.raises(LacError):
        list(AC(Wide(2), 16).to_bin.run([0]))
    with pytest.raises(LacError):
        list(AC(Wide(2), 16).from_bin.run([1, 0, 1]))
