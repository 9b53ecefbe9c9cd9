"""Host check of the kernels' per-stream arithmetic (lac_core.h) against the oracle.

Compiles tests/native/core_check.cpp (host code only) with hipcc; no GPU needed.
"""
import ctypes as C
import os
import random
import subprocess

import numpy as np
import pytest

from conftest import REPO, load_golden
from lac_amd import synth
from oracle import oracle as coracle

SO = os.path.join(REPO, "tests", "native", "libcorecheck.so")
SRC = os.path.join(REPO, "tests", "native", "core_check.cpp")


@pytest.fixture(scope="module")
def core():
    deps = [SRC] + [os.path.join(REPO, "lac_amd", "csrc", h) for h in ("lac_core.h", "lac_hc.h")] + [
        os.path.join(REPO, "include", "lac.h")]
    if not os.path.exists(SO) or os.path.getmtime(SO) < max(os.path.getmtime(d) for d in deps):
        subprocess.run(["hipcc", "-O2", "-std=c++17", "-fPIC", "-shared", "-I", os.path.join(REPO, "lac_amd", "csrc"),
                        "-I", os.path.join(REPO, "include"), SRC, "-o", SO], check=True)
    lib = C.CDLL(SO)
    lib.cc_div_floor.restype = C.c_uint64
    lib.cc_div_floor.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]
    lib.cc_div_floor_inv.restype = C.c_uint64
    lib.cc_div_floor_inv.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]
    lib.cc_encode.restype = C.c_int
    lib.cc_encode.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_int64, C.c_int64, C.c_void_p, C.c_int,
                              C.c_void_p, C.c_uint64, C.c_void_p]
    return lib


def _enc(core, rows, syms, prec):
    a = np.ascontiguousarray(rows)
    s = np.ascontiguousarray(np.asarray(syms, dtype=np.int32))
    cap = (len(s) * (prec + 2) + 256) // 8 * 8
    out = np.zeros(cap, dtype=np.uint8)
    nb = np.zeros(1, dtype=np.uint64)
    stride = 0 if a.shape[0] == 1 else a.shape[1]
    rc = core.cc_encode(a.ctypes.data, a.itemsize, a.shape[1], len(s), stride, s.ctypes.data, prec,
                        out.ctypes.data, cap, nb.ctypes.data)
    L = int(nb[0])
    return rc, out[:(L + 7) // 8].tobytes(), L


def test_div_floor_exact(core):
    rng = random.Random(5)
    for _ in range(20000):
        d = rng.choice([1, 2, 3, rng.randrange(1, 1 << 20), rng.randrange(1, 1 << 47), rng.randrange(1, 1 << 64)])
        q = rng.randrange(0, 1 << rng.choice([8, 32, 47, 61, 62, 63, 64]))
        r = rng.randrange(0, d)
        N = q * d + r
        if N >> 128:
            continue
        assert core.cc_div_floor(N >> 64, N & ((1 << 64) - 1), d) == q
        assert core.cc_div_floor_inv(N >> 64, N & ((1 << 64) - 1), d) == q


def test_frac_mul_div_exact(core):
    """The split-path coder step's row-fraction division (lac_core.h frac_mul_div)
    against exact big-int floor/ceil, including c == T, c == 0 and T near 2^63."""
    core.cc_frac_mul_div.restype = C.c_uint64
    core.cc_frac_mul_div.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_int]
    rng = random.Random(11)
    for i in range(40000):
        T = rng.choice([1, 2, 3, rng.randrange(1, 1 << 20), rng.randrange(1, 1 << 40), rng.randrange(1, 1 << 63),
                        (1 << 63) - rng.randrange(1, 1000)])
        c = rng.choice([0, T, rng.randrange(0, T + 1), T - 1 if T > 1 else 0])
        prec = rng.randint(2, 61)
        w = rng.randrange((1 << (prec - 1)) + 1, (1 << prec) + 1)
        ceil = i & 1
        want = -(-(c * w) // T) if ceil else (c * w) // T
        assert core.cc_frac_mul_div(c, w, T, ceil) == want, (c, w, T, ceil)
    assert core.cc_frac_mul_div(5, 1 << 47, 1 << 63, 1) == (1 << 64) - 1     # T >= 2^63: no fraction


def test_frac_mul_div_uniform_form_exact(core):
    """frac_mul_div<true> (k_encode's compare-free form: sign masks of r - T and r - 2T)
    against exact big-int floor/ceil for T < 2^62, edges included (T just below 2^62,
    c == T, c == 0, w at both ends of its range)."""
    f = core.cc_frac_mul_div_uni
    f.restype = C.c_uint64
    f.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_int]
    rng = random.Random(12)
    for i in range(60000):
        T = rng.choice([1, 2, 3, rng.randrange(1, 1 << 20), rng.randrange(1, 1 << 40), rng.randrange(1, 1 << 62),
                        (1 << 62) - rng.randrange(1, 1000), (1 << 61) + rng.randrange(0, 1000)])
        c = rng.choice([0, T, rng.randrange(0, T + 1), T - 1 if T > 1 else 0, 1 if T >= 1 else 0])
        prec = rng.randint(2, 61)
        w = rng.choice([(1 << (prec - 1)) + 1, 1 << prec, rng.randrange((1 << (prec - 1)) + 1, (1 << prec) + 1)])
        ceil = i & 1
        want = -(-(c * w) // T) if ceil else (c * w) // T
        assert f(c, w, T, ceil) == want, (c, w, T, ceil)
    assert f(5, 1 << 47, 1 << 62, 1) == (1 << 64) - 1                         # T >= 2^62: not this form


def test_frac_mul_div32_exact(core):
    """frac_mul_div32 (k_encode's straight block: 32-bit counts and totals, the
    remainder's products in 32 x 64 bits) against exact big-int floor/ceil, edges
    included (T = 1 and just below 2^32, c == T, c == 0, w at both ends of its range)."""
    f = core.cc_frac_mul_div32
    f.restype = C.c_uint64
    f.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_int]
    rng = random.Random(13)
    for i in range(60000):
        T = rng.choice([1, 2, 3, rng.randrange(1, 1 << 20), rng.randrange(1, 1 << 32), (1 << 32) - rng.randrange(1, 1000),
                        (1 << 31) + rng.randrange(0, 1 << 20)])
        c = rng.choice([0, T, rng.randrange(0, T + 1), T - 1 if T > 1 else 0, 1])
        c = min(c, T)
        prec = rng.randint(2, 61)
        w = rng.choice([(1 << (prec - 1)) + 1, 1 << prec, rng.randrange((1 << (prec - 1)) + 1, (1 << prec) + 1)])
        ceil = i & 1
        want = -(-(c * w) // T) if ceil else (c * w) // T
        assert f(c, w, T, ceil) == want, (c, w, T, ceil)
    assert f(5, 1 << 47, 1 << 32, 1) == (1 << 64) - 1                         # T >= 2^32: not this form


def test_div_small_exact(core):
    """div_small (the decode step's quotient at prec <= 50 / totals < 2^50): exact
    floor((n*m + add)/d) for quotients below 2^50, with the reciprocal up to 2^-49
    off (the device's v_rcp_f64 after one Newton step is good to ~2^-50)."""
    import random
    core.cc_div_small.restype = C.c_uint64
    core.cc_div_small.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_double]
    core.cc_div_small_mask.restype = C.c_uint64          # the sign-mask correction (div_small_fix_mask)
    core.cc_div_small_mask.argtypes = core.cc_div_small.argtypes
    rng = random.Random(11)
    n_cases = 0
    while n_cases < 40000:
        d = rng.randint(1, (1 << rng.randint(1, 50)))
        n = rng.randint(0, (1 << rng.randint(0, 50)))
        m = rng.randint(0, (1 << rng.randint(0, 50)))
        add = rng.choice([0, d - 1, rng.randint(0, d)])
        q = (n * m + add) // d
        if q >= 1 << 50:
            continue
        rel = rng.choice([0.0, 2.0 ** -49, -2.0 ** -49, rng.uniform(-1, 1) * 2.0 ** -50])
        assert core.cc_div_small(n, m, add, d, rel) == q, (n, m, add, d, rel)
        assert core.cc_div_small_mask(n, m, add, d, rel) == q, (n, m, add, d, rel)
        n_cases += 1
    # the decoder's own shapes: targets floor(v*T/w), v < w, and ranges ceil(c*w/T), c <= T
    for _ in range(20000):
        prec = rng.randint(2, 50)
        w = rng.randint((1 << (prec - 1)) + 1, 1 << prec)
        T = rng.randint(1, (1 << 50) - 1)
        v = rng.randint(0, w - 1)
        c = rng.randint(0, T)
        assert core.cc_div_small(v, T, 0, w, 2.0 ** -50) == v * T // w
        assert core.cc_div_small(c, w, T - 1, T, -2.0 ** -50) == -(-(c * w) // T)
        assert core.cc_div_small_mask(v, T, 0, w, 2.0 ** -50) == v * T // w
        assert core.cc_div_small_mask(c, w, T - 1, T, -2.0 ** -50) == -(-(c * w) // T)


def test_div_mid_exact(core):
    """div_mid (the lean decode step's ranges on u64 rows with totals of 2^50 and more):
    exact floor((n*m + add)/d) for quotients up to 2^50 with d anywhere below 2^64, from
    one estimate and the 128-bit remainder -- random, power-of-two-edge and the decoder's
    own shapes ceil(c*w/T), c <= T < 2^64, w <= 2^50."""
    import random
    core.cc_div_mid.restype = C.c_uint64
    core.cc_div_mid.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64]
    rng = random.Random(12)
    n_cases = 0
    while n_cases < 40000:
        d = rng.randint(1, (1 << rng.randint(1, 64)) - 1)
        m = rng.randint(0, 1 << rng.randint(0, 51))
        n = rng.randint(0, (1 << rng.randint(0, 64)) - 1)
        add = rng.choice([0, d - 1, rng.randint(0, d - 1)])
        q = (n * m + add) // d
        if q > 1 << 50:
            continue
        assert core.cc_div_mid(n, m, add, d) == q, (n, m, add, d)
        n_cases += 1
    for _ in range(40000):
        prec = rng.randint(2, 50)
        w = rng.randint((1 << (prec - 1)) + 1, 1 << prec)
        T = rng.choice([rng.randint(1 << 50, (1 << 64) - 1), (1 << 64) - 1, (1 << 63) + rng.randint(0, 99),
                        rng.randint(1, (1 << 64) - 1)])
        c = rng.choice([rng.randint(0, T), T, T - 1, 0, 1])
        assert core.cc_div_mid(c, w, T - 1, T) == -(-(c * w) // T), (c, w, T)
        assert core.cc_div_mid(c, w, 0, T) == c * w // T, (c, w, T)


def test_div_mid_w_exact(core):
    """div_mid_est_w (the lean step's wide ranges: m through the 2^52 magic, the estimate
    rounded by it, the ceil mapping's addend T - 1 passed as T rounded to a double): exact
    floor((n*m + add)/d) for quotients up to 2^50 -- random addends passed exactly, and the
    decoder's shapes ceil(c*w/T) with T >= 2^50, c <= T, w <= 2^50."""
    import random
    core.cc_div_mid_w.restype = C.c_uint64
    core.cc_div_mid_w.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_double, C.c_uint64]
    rng = random.Random(13)
    n_cases = 0
    while n_cases < 40000:
        d = rng.randint(1, (1 << rng.randint(1, 64)) - 1)
        m = rng.randint(0, 1 << rng.randint(0, 51))
        n = rng.randint(0, (1 << rng.randint(0, 64)) - 1)
        add = rng.choice([0, d - 1, rng.randint(0, d - 1)])
        q = (n * m + add) // d
        if q > 1 << 50:
            continue
        assert core.cc_div_mid_w(n, m, add, float(add), d) == q, (n, m, add, d)
        n_cases += 1
    for _ in range(40000):
        prec = rng.randint(2, 50)
        w = rng.randint((1 << (prec - 1)) + 1, 1 << prec)
        T = rng.choice([rng.randint(1 << 50, (1 << 64) - 1), (1 << 64) - 1, (1 << 63) + rng.randint(0, 99),
                        (1 << 50) + rng.randint(0, 99)])
        c = rng.choice([rng.randint(0, T), T, T - 1, 0, 1])
        assert core.cc_div_mid_w(c, w, T - 1, float(T), T) == -(-(c * w) // T), (c, w, T)
        assert core.cc_div_mid_w(c, w, 0, 0.0, T) == c * w // T, (c, w, T)


def test_div_near_exact(core):
    """div_near (the lean decode step's rows below 2^50, two sign tests): u32 rows' targets
    floor(v*T/w), T < 2^32, with the reciprocal of w up to 16 ulps off (the device's
    v_rcp_f64 + Newton is good to ~11), and the ranges ceil(c*w/T), c <= T < 2^32, with
    the correctly rounded 1/T the stats pass stores -- prec 2..50, adversarial and random."""
    import random
    core.cc_div_near.restype = C.c_uint64
    core.cc_div_near.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, C.c_int]
    rng = random.Random(13)
    for _ in range(60000):
        prec = rng.randint(2, 50)
        w = rng.choice([rng.randint((1 << (prec - 1)) + 1, 1 << prec), 1 << prec, (1 << (prec - 1)) + 1])
        T = rng.choice([rng.randint(1, (1 << 32) - 1), (1 << 32) - 1, rng.randint(1, 1 << 16), 1])
        v = rng.choice([rng.randint(0, w - 1), w - 1, 0])
        ulps = rng.choice([0, 16, -16, rng.randint(-16, 16)])
        assert core.cc_div_near(v, T, 0, w, ulps, 0) == v * T // w, (v, T, w, ulps)
        c = rng.choice([rng.randint(0, T), T, T - 1, 0, 1])
        assert core.cc_div_near(c, w, T - 1, T, 0, 1) == -(-(c * w) // T), (c, w, T)
        assert core.cc_div_near(c, w, 0, T, 0, 1) == c * w // T, (c, w, T)
    # u64 rows below 2^50: targets with 1/w within 1 ulp (recip2), ranges with 1/T exact
    for _ in range(60000):
        prec = rng.randint(2, 50)
        w = rng.choice([rng.randint((1 << (prec - 1)) + 1, 1 << prec), 1 << prec, (1 << (prec - 1)) + 1])
        T = rng.choice([rng.randint(1, (1 << 50) - 1), (1 << 50) - 1, rng.randint(1 << 32, 1 << 50)])
        v = rng.choice([rng.randint(0, w - 1), w - 1, 0])
        ulps = rng.choice([0, 1, -1])
        assert core.cc_div_near(v, T, 0, w, ulps, 0) == v * T // w, (v, T, w, ulps)
        c = rng.choice([rng.randint(0, T), T, T - 1, 0, 1])
        assert core.cc_div_near(c, w, T - 1, T, 0, 0) == -(-(c * w) // T), (c, w, T)


def test_core_matches_golden(core):
    for kind in ("static", "perstep"):
        for c in load_golden("small_cases.json")[kind]:
            if not c["syms"]:
                continue
            rows = np.array(c["rows"], dtype=np.uint32)
            rc, data, L = _enc(core, rows, c["syms"], c["prec"])
            assert rc == 0 and L == c["L"] and data.hex() == c["bytes"], c
    for c in load_golden("gen_cases.json"):
        rows = np.stack([synth.pmf_row(c["seed"], t, 0, c["V"], c["kind"], c["exp_range"]) for t in range(c["steps"])])
        rc, data, L = _enc(core, rows, c["syms"], c["prec"])
        assert rc == 0 and L == c["L"] and data.hex() == c["bytes"], c["name"]


@pytest.mark.parametrize("seed", range(6))
def test_core_random_vs_oracle(core, seed):
    rng = random.Random(100 + seed)
    for _ in range(60):
        V = rng.choice([2, 3, 7, 64, 300, 1000])
        prec = rng.randint(max(2, (V - 1).bit_length() + 1), 61)
        kind = rng.choice(["loguniform", "zeros", "peaked", "flat", "llama64"])
        steps = rng.randint(1, 40)
        pmf, sym = synth.make_batch(rng.randrange(1 << 30), steps, 1, V, kind)
        rows = pmf[:, 0, :]
        want = coracle.encode(rows, sym[:, 0], prec)
        rc, data, L = _enc(core, rows, sym[:, 0], prec)
        assert rc == 0 and (data, L) == want[:2], (V, prec, kind)


def test_div_floor_inv_with_an_inexact_reciprocal(core):
    """The device's div_floor_inv estimates with v_rcp_f64, an approximation of 1/d
    (lac_core.h recip).  With the reciprocal up to 4 ULPs off the correctly rounded
    one (tools/rcp_probe.hip measures the hardware's own error on the MI355X) the
    quotient stays exact and the final correction loops run at most twice."""
    core.cc_div_floor_inv_ulp.restype = C.c_uint64
    core.cc_div_floor_inv_ulp.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, C.POINTER(C.c_int)]
    rng = random.Random(17)
    worst = 0
    fix = C.c_int()
    for i in range(60000):
        d = rng.choice([1, 3, rng.randrange(1, 1 << 20), rng.randrange(1, 1 << 47), rng.randrange(1, 1 << 64),
                        (1 << 64) - rng.randrange(1, 1 << 10), (1 << 63) + rng.randrange(0, 1 << 10)])
        q = rng.choice([rng.randrange(0, 1 << 64), (1 << 64) - 1 - rng.randrange(0, 1 << 12), rng.randrange(0, 1 << 48)])
        r = rng.randrange(0, d)
        N = q * d + r
        if N >> 128:
            continue
        ulps = rng.choice([-4, -2, -1, 0, 1, 2, 4])
        got = core.cc_div_floor_inv_ulp(N >> 64, N & ((1 << 64) - 1), d, ulps, C.byref(fix))
        assert got == q, (N, d, ulps)
        worst = max(worst, fix.value)
    assert worst <= 2, worst


def test_cr_ratio_is_pythons_division(core):
    """lac_core.h cr_ratio == CPython's int / int (correctly rounded) -- the float
    A_from_bin.flush ranks candidates by (arith_code.py:305-312)."""
    import struct
    core.cc_cr_ratio.restype = C.c_uint64
    core.cc_cr_ratio.argtypes = [C.c_uint64, C.c_uint64]
    rng = random.Random(23)
    for i in range(60000):
        b = rng.choice([1, 2, 3, rng.randrange(1, 1 << 20), rng.randrange(1, 1 << 53), rng.randrange(1 << 53, 1 << 63),
                        (1 << 62) + rng.randrange(0, 1 << 8)])
        a = rng.choice([0, b, b - 1, rng.randrange(0, b + 1), b // 2, b // 3 + 1])
        a = max(0, min(a, b))
        want = struct.unpack("<Q", struct.pack("<d", a / b))[0]
        assert core.cc_cr_ratio(a, b) == want, (a, b)


def test_host_arithmetic_and_oracle_under_sanitizers():
    """AddressSanitizer + UndefinedBehaviorSanitizer build of the kernels' host-side
    arithmetic (lac_core.h via core_check.cpp) and the C oracle, cross-checked on
    seeded random inputs by tests/native/sanitize_main.cpp (make -C tests/native asan)."""
    native = os.path.join(REPO, "tests", "native")
    subprocess.run(["make", "-s", "-C", native, "asan"], check=True)
    r = subprocess.run([os.path.join(native, "_asan", "sanitize_check")], capture_output=True, text=True, timeout=600)
    report = r.stdout + r.stderr
    assert r.returncode == 0, report[-3000:]
    assert "sanitize_main: ok" in report
    assert "runtime error" not in report and "AddressSanitizer" not in report
