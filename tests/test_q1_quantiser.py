"""The q1 logits quantiser: C oracle vs an independent numpy restatement (CPU)."""
import re

import numpy as np
import pytest

from conftest import REPO
from oracle import oracle as coracle
from oracle import restate


def _tab():
    src = open(f"{REPO}/include/lac_q1_table.h").read()
    return [int(x) for x in re.findall(r"(\d+)u", src.split("LAC_Q1_TAB_INIT")[1])]


def _bf16(x):
    """float32 -> bf16 bit patterns (round to nearest even) as uint16."""
    u = np.asarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) >> 16
    return u.astype(np.uint16)


def _widen(b):
    return (b.astype(np.uint32) << 16).view(np.float32)


def test_table_is_exact_exp():
    import math
    tab = _tab()
    assert len(tab) == 17 * 32 + 1 and tab[0] == 1 << 24 and tab[-1] >= 1
    for i in (1, 31, 100, 311, 500, 544):
        assert abs(tab[i] - 2 ** 24 * math.exp(-i / 32)) <= 0.5 + 1e-9 * tab[i]


@pytest.mark.parametrize("V,prec", [(32000, 48), (128256, 48), (1000, 40), (17, 24)])
def test_c_oracle_matches_numpy_restatement(V, prec):
    tab = _tab()
    rng = np.random.default_rng(V + prec)
    for scale in (0.5, 3.0, 40.0):
        x = (rng.standard_normal(V) * scale).astype(np.float32)
        b = _bf16(x)
        got_b = coracle.q1_quantize(b, prec)
        want_b = restate.q1_quantize(_widen(b), prec, tab)
        assert (got_b == want_b).all()
        got_f = coracle.q1_quantize(x, prec)
        want_f = restate.q1_quantize(x, prec, tab)
        assert (got_f == want_f).all()
        k = min(24, prec - 1 - (V - 1).bit_length())
        assert got_f.max() == 1 << k and got_f.min() >= 1
        assert int(got_f.astype(np.uint64).sum()) <= V << k       # never fudged: T <= 2^(prec-1)


def test_non_finite_logits():
    tab = _tab()
    x = np.array([0.0, -np.inf, np.nan, 5.0, -1e30, 1e-40], dtype=np.float32)
    got = coracle.q1_quantize(x, 48)
    assert (got == restate.q1_quantize(x, 48, tab)).all()
    assert got[3] == 1 << 24 and got[1] == 1 and got[2] == 1
    allinf = np.full(8, -np.inf, dtype=np.float32)
    assert (coracle.q1_quantize(allinf, 48) == 1).all()


def test_library_q1_k_matches_oracle():
    """lac_q1_k (host-only C-ABI function, no GPU needed) == the oracle's k."""
    from lac_amd import _lib
    L = _lib.load()
    for prec in (22, 24, 32, 40, 48, 61):
        for V in (1, 2, 3, 24, 1000, 1024, 1025, 32000, 128256, 1 << 20):
            if (1 << (prec - 1)) >= V:
                assert L.lac_q1_k(prec, V) == coracle.lib().lacref_q1_k(prec, V), (prec, V)


def test_extreme_rows_exact_fma():
    """Rows whose fma sum is not exact in float64 (tiny logits next to a large max,
    maxima around the GPU fast-path bound 2^18): C fmaf == exact rounding."""
    tab = _tab()
    rng = np.random.default_rng(9)
    for m in (3.0e5, 2.0 ** 18, 2.0 ** 18 - 0.5, -2.0 ** 18, 1.5e30, 17.0):
        x = (np.float32(m) - np.abs(rng.standard_normal(64)).astype(np.float32) * np.float32(5)).astype(np.float32)
        if m > 0:
            x[:8] = np.float32(1e-30) * np.arange(1, 9, dtype=np.float32)
        x[8] = m
        x[9] = np.float32(m) - np.float32(17.0)
        x[10] = np.float32(m) - np.float32(1 / 64)
        x[11] = -np.float32(1e38)
        got = coracle.q1_quantize(x, 48)
        assert (got == restate.q1_quantize(x, 48, tab)).all(), m
        if abs(m) < 2 ** 20:                  # beyond ~2^24, c = RNE(544 - 32m) drops the 544: all-ones table
            assert got.max() == got[8] == 1 << 24
        else:
            assert (got >= 1).all()
