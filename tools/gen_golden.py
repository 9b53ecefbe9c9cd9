#!/usr/bin/env python3
"""Generate golden vectors by running the REFERENCE coder (this container only).

    PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py [--kat]

Imports /root/reference (read-only, never copied) and records, for integer
tables regenerated from ``lac_amd.synth`` parameters or stored inline, what the
reference produces:

* ``A_to_bin.run(syms)`` raw carry digits, per-symbol digit trace (small cases)
* ``A_to_bin.encode(syms)`` -> (R, L) and ``bytes(group_bits(bits(syms)))``
  (the ``measure_compress`` byte format, arith_code.py:401-420)
* ``A_from_bin.run(bits, stop=0)`` decoded symbols (how many it determines)
* KAT-1 / KAT-2 hashes with ``--kat`` (~2 minutes)

Per-step tables use a Replay predictor: a CDFPredictor
whose ``accept`` advances to the next row; rows past the end repeat the last.
Output: tests/golden/*.json (data only: inputs and expected outputs).
"""
from __future__ import annotations

import argparse
import hashlib
import itertools
import json
import os
import random
import sys
import time

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, "/root/reference")

import numpy as np  # noqa: E402

import arith_code as ref  # noqa: E402  (the reference, read-only)
from lac_amd import synth  # noqa: E402

GOLDEN = os.path.join(REPO, "tests", "golden")


class Replay(ref.CDFPredictor):
    def __init__(self, rows):
        self.rows = rows
        self.i = 0
        self._load()

    def _load(self):
        r = self.rows[min(self.i, len(self.rows) - 1)]
        self.dist = list(itertools.accumulate(int(v) for v in r))
        self.minp = min(filter(lambda v: v > 0, self.pdf_iter))

    def accept(self, symbol):
        self.i += 1
        self._load()

    def copy(self):
        return Replay(self.rows)


def run_reference(rows, syms, prec, want_trace=True, want_decode=True):
    ac = ref.AC(Replay(rows), prec)
    enc = ac.to_bin
    trace = []
    if want_trace:
        for s in syms:
            trace.append(list(enc.step(s)))
        flush = list(enc.flush())
    R, L = ac.to_bin.encode(syms)
    bits = list(ac.to_bin.bits(syms))
    assert len(bits) == L and all(b in (0, 1) for b in bits)
    assert int("".join(map(str, bits)) or "0", 2) == R
    data = bytes(ref.group_bits(iter(bits)))
    rec = {"L": L, "bytes": data.hex()}
    if want_trace:
        digits = [d for st in trace for d in st] + flush
        assert sum(d << (L - 1 - k) for k, d in enumerate(digits)) == R
        rec["trace"] = trace
        rec["flush"] = flush
    if want_decode:
        dec = list(ac.from_bin.run(iter(bits), stop=0))
        assert dec[:len(syms)] == list(syms), "reference round trip failed"
        rec["decoded_count"] = len(dec)
        rec["decoded_extra"] = dec[len(syms):]
    return rec


def small_cases(rng, n, perstep):
    out = []
    while len(out) < n:
        V = rng.randint(2, 12)
        prec = rng.randint(max(2, (V - 1).bit_length() + 1), 20)
        choices = [0, 1, 1, 2, 3, 5, 8, 100, 1000, 100000]
        T = rng.randint(0, 10)
        nrows = T if perstep and T > 0 else 1
        rows = []
        for _ in range(nrows):
            pmf = [rng.choice(choices) for _ in range(V)]
            while sum(1 for p in pmf if p > 0) < 2:      # a one-symbol row makes the
                pmf[rng.randrange(V)] = rng.choice(choices[1:])  # bit-driven reference
            rows.append(pmf)                                     # decoder loop forever
        syms = []
        for t in range(T):
            r = rows[min(t, nrows - 1)]
            syms.append(rng.choice([i for i in range(V) if r[i] > 0]))
        rec = {"V": V, "prec": prec, "rows": rows, "syms": syms}
        rec.update(run_reference(rows, syms, prec))
        out.append(rec)
    return out


GEN_CASES = [
    # (name, seed, kind, exp_range, V, steps, prec, trace, decode)
    ("lu17_p16", 11, "loguniform", 8, 17, 64, 16, True, True),
    ("lu256_p24", 12, "loguniform", 16, 256, 64, 24, True, True),
    ("zeros256_p32", 13, "zeros", 24, 256, 48, 32, True, True),
    ("lu1000_p48", 14, "loguniform", 24, 1000, 40, 48, True, True),
    ("peak1000_p61", 15, "peaked", 24, 1000, 40, 61, True, True),
    ("flat300_p10", 16, "flat", 24, 300, 64, 10, True, True),       # mixed fudged/unfudged
    ("lu1000_p16", 17, "loguniform", 24, 1000, 24, 16, True, True),  # fudged
    ("lu32000_p48", 18, "loguniform", 24, 32000, 12, 48, True, True),
    ("peak32000_p48", 19, "peaked", 24, 32000, 12, 48, True, True),
    ("zeros32000_p40", 20, "zeros", 24, 32000, 8, 40, True, True),
    ("lu32000_p24", 21, "loguniform", 24, 32000, 4, 24, True, False),  # fudged, big V
    ("llama64_1000_p48", 22, "llama64", 0, 1000, 16, 48, True, True),  # u64, fudged
    ("llama64_32000_p48", 23, "llama64", 0, 32000, 3, 48, True, False),
    ("lu5000_p61", 24, "loguniform", 24, 5000, 16, 61, True, True),
]


# Round 6: cases that reach each straight 64-step form of the split-path encoder
# (lac_encode.hip k_encode) when coded untraced -- u32 tables with every total below both
# 2^32 and 2^(prec-1) (the u32 form), and 32-bit totals above 2^(prec-1) (the u64 kernel's
# T32 + FT form once stored as u64: every row can fudge at prec 21, some at prec 31) --
# with full 64-step blocks and a part-filled last one.
STRAIGHT_CASES = [
    ("u32s_lu1000_p48", 31, "loguniform", 16, 1000, 150, 48, True, True),
    ("u32s_lu32000_p40", 32, "loguniform", 11, 32000, 70, 40, True, False),
    ("t32ft_lu1000_p21", 33, "loguniform", 16, 1000, 140, 21, True, True),
    ("t32ft_lu1000_p31", 34, "loguniform", 18, 1000, 140, 31, True, True),
    ("t32ft_flat300_p10", 35, "flat", 24, 300, 130, 10, True, True),
]


def gen_case(name, seed, kind, er, V, steps, prec, trace, decode):
    rows = [synth.pmf_row(seed, t, 0, V, kind, er or 24) for t in range(steps)]
    syms = [synth.sample_symbol(r, seed, t, 0) for t, r in enumerate(rows)]
    t0 = time.time()
    rec = {"name": name, "seed": seed, "kind": kind, "exp_range": er or 24, "V": V,
           "steps": steps, "prec": prec, "syms": syms}
    rec.update(run_reference(rows, syms, prec, trace, decode))
    print(f"  {name}: L={rec['L']} ({time.time() - t0:.1f}s)", flush=True)
    return rec


def kat1():
    """KAT-1: A_to_bin + CDFPredictor(range(1,257)) @48 is the identity on bytes."""
    data = np.random.default_rng(0).integers(0, 256, 2 ** 20, dtype=np.uint8).tobytes()
    ac = ref.AC(ref.CDFPredictor(list(range(1, 257))), 48)
    t0 = time.time()
    out = bytes(ref.group_bits(ac.to_bin.bits(iter(data))))
    t1 = time.time()
    dec = list(ac.from_bin.run(ref.ungroup_bits(out), stop=0))
    t2 = time.time()
    assert bytes(dec[:len(data)]) == data
    return {"n": len(data), "in_sha256": hashlib.sha256(data).hexdigest(),
            "out_sha256": hashlib.sha256(out).hexdigest(), "out_len": len(out),
            "identity": out == data, "ref_encode_s": t1 - t0, "ref_decode_s": t2 - t1}


def kat2(nbytes):
    """KAT-2: ACSampler(48) uniform-256 encode."""
    import arithmetic_coding as acd
    data = np.random.default_rng(0).integers(0, 256, nbytes, dtype=np.uint8).tobytes()
    out = bytearray()
    s = acd.ACSampler(48)
    s.compress_tokens = iter(data)
    s.compress_output = acd.packbits(out.append)

    def done():
        s.on_compress_done = None
        s.flush_compress()
        s.compress_output.flush()
        s.compress_output = None
    s.on_compress_done = done
    t0 = time.time()
    while not s.compress_done:
        s.sample(np.ones(256))
    return {"n": nbytes, "in_sha256": hashlib.sha256(data).hexdigest(),
            "out_sha256": hashlib.sha256(bytes(out)).hexdigest(), "out_len": len(out),
            "out_tail_hex": bytes(out[-8:]).hex(), "ref_s": time.time() - t0,
            "out_hex": bytes(out).hex() if nbytes <= 4096 else None}


def acsampler_nonuniform(rng):
    """ACSampler on a non-uniform float pdf: record the uint64 cdf it builds + bits."""
    import arithmetic_coding as acd
    cases = []
    for k in range(6):
        V = rng.choice([3, 10, 256, 1000])
        pdf = np.array([rng.random() ** 3 * 100 + 1e-9 for _ in range(V)], dtype=np.float64)
        toks = [rng.randrange(V) for _ in range(rng.randint(1, 200))]
        s = acd.ACSampler(48)
        p = np.array(pdf, dtype=np.float64)
        p += s.get_lop_bias(p)
        p *= s.region.one / np.sum(p)
        cdf = np.cumsum(p).astype(np.uint64)
        bits = []
        s.compress_tokens = iter(toks)
        s.compress_output = bits.append

        def done(s=s):
            s.on_compress_done = None
            s.flush_compress()
            s.compress_output = None
        s.on_compress_done = done
        while not s.compress_done:
            s.sample(pdf)
        cases.append({"cdf": [int(c) for c in cdf], "tokens": toks, "bits": "".join(map(str, bits))})
    return cases


def acsampler_callbacks(seed=20261016):
    """ACSampler with a different float pdf per token: the bits, every
    bits_per_token value (Region.entropy_of at the current span) and the
    unencodable-token assertion (arithmetic_coding.py:73-95, :155-157)."""
    import arithmetic_coding as acd
    rng = np.random.default_rng(seed)
    cases = []
    for k in range(5):
        V = int(rng.choice([2, 7, 256, 1000]))
        n = int(rng.integers(1, 120))
        pdfs = [(rng.random(V) ** 4 * 50 + 1e-12).tolist() for _ in range(n)]
        toks = [int(rng.integers(0, V)) for _ in range(n)]
        s = acd.ACSampler(48)
        bits, ent = [], []
        s.compress_tokens = iter(toks)
        s.compress_output = bits.append
        s.bits_per_token = ent.append

        def done(s=s):
            s.on_compress_done = None
            s.flush_compress()
            s.compress_output = None
        s.on_compress_done = done
        i = 0
        while not s.compress_done:
            s.sample(pdfs[min(i, n - 1)])
            i += 1
        # the phantom token after exhaustion also reports an entropy: keep the
        # per-token values of the real tokens only
        cases.append({"pdfs": pdfs, "tokens": toks, "bits": "".join(map(str, bits)), "entropy": ent[:n]})
    # scaled cdfs the reference rejects: a token whose floor-mapped width is 0
    bad = []
    for cdf, pre in (([1, 2, 1 << 48], []), ([1, 2, 1 << 50], []), ([5, 5, 9], []),
                     ([1 << 40, (1 << 40) + 1, 1 << 48], [1, 2]), ([1 << 40, (1 << 40) + 1, 1 << 48], [1, 1, 2]),
                     ([1, 2, 1 << 48], [0, 1]), ([1, 2, 1 << 48], [2, 0, 1])):
        s = acd.ACSampler(48)
        s.compress_tokens = iter(pre + [0])
        s.compress_output = lambda b: None
        good = np.array([3 << 44, 7 << 44, 10 << 44], dtype=np.uint64)
        for t in pre:
            s.sample_scaled_cdf(good)
        try:
            s.sample_scaled_cdf(np.array(cdf, dtype=np.uint64))
            bad.append({"cdf": cdf, "pre": pre, "raises": None})
        except AssertionError as e:
            bad.append({"cdf": cdf, "pre": pre, "raises": str(e)})
    return {"cases": cases, "unencodable": bad}


def deterministic():
    """Rows with a single positive entry: the encoder emits nothing for them."""
    out = []
    for rows, syms, prec in (([[1000, 0]], [0, 0, 0], 16), ([[0, 0, 7, 0]], [2] * 5, 12),
                             ([[5, 3], [0, 9], [4, 4]], [1, 1, 0], 10)):
        rec = {"rows": rows, "syms": syms, "prec": prec}
        rec.update(run_reference(rows, syms, prec, want_decode=False))
        out.append(rec)
    return out


def ternary():
    ac = ref.AC()
    return {"syms": [1, 1, 2], "digits": list(ac.to_bin.run([1, 1, 2])),
            "encode": list(ac.to_bin.encode([1, 1, 2])), "bits": list(ac.to_bin.bits([1, 1, 2])),
            "decoded": list(ac.from_bin.run([1, 0, 0, 0, 1, 0], stop=0))}


def errors():
    cdf = [1, 3, 6, 10]
    out = {}
    try:
        list(ref.AC(ref.CDFPredictor(cdf), 16).to_bin.run([0, 4]))
    except AssertionError as e:
        out["symbol_range"] = [str(a) for a in e.args]
    try:
        list(ref.AC(ref.CDFPredictor(cdf), 16).to_bin.run([-1]))
    except AssertionError as e:
        out["symbol_negative"] = [str(a) for a in e.args]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kat", action="store_true", help="also run the 1 MiB KATs (~2 min)")
    ap.add_argument("--only", choices=["acsampler_cb", "straight"], help="write just this fixture file")
    a = ap.parse_args()
    os.makedirs(GOLDEN, exist_ok=True)
    if a.only == "straight":
        with open(os.path.join(GOLDEN, "straight_cases.json"), "w") as f:
            json.dump([gen_case(*c) for c in STRAIGHT_CASES], f, separators=(",", ":"))
        return
    if a.only == "acsampler_cb":
        with open(os.path.join(GOLDEN, "acsampler_cb.json"), "w") as f:
            json.dump(acsampler_callbacks(), f, separators=(",", ":"))
        return
    rng = random.Random(20261015)
    small = {"static": small_cases(rng, 250, perstep=False),
             "perstep": small_cases(rng, 250, perstep=True)}
    with open(os.path.join(GOLDEN, "small_cases.json"), "w") as f:
        json.dump(small, f, separators=(",", ":"))
    print("small cases done", flush=True)
    gen = [gen_case(*c) for c in GEN_CASES]
    with open(os.path.join(GOLDEN, "gen_cases.json"), "w") as f:
        json.dump(gen, f, separators=(",", ":"))
    misc = {"ternary": ternary(), "errors": errors(), "deterministic": deterministic(),
            "acsampler_small": kat2(1000), "acsampler_nonuniform": acsampler_nonuniform(rng)}
    with open(os.path.join(GOLDEN, "misc.json"), "w") as f:
        json.dump(misc, f, indent=1)
    if a.kat:
        kats = {"kat1": kat1()}
        print("kat1", kats["kat1"], flush=True)
        kats["kat2"] = kat2(2 ** 20)
        print("kat2", {k: v for k, v in kats["kat2"].items() if k != "out_hex"}, flush=True)
        with open(os.path.join(GOLDEN, "kat.json"), "w") as f:
            json.dump(kats, f, indent=1)


if __name__ == "__main__":
    main()
