#!/usr/bin/env python3
"""Speed of the drop-in surface (AC / A_to_bin / A_from_bin) at V=32000 (VERDICT r3
item 3), the coders a reference user switches to unchanged (arith_code.py:76-155).

    python tools/dropin_bench.py [--n 10000] [--out gpurun_out/dropin.json]

* static CDFPredictor (accept is the base no-op): ``AC(p, 48).to_bin.encode(syms)``
  and ``from_bin.run(bits, stop=0)`` on n symbols drawn from the table;
* a ProbPredictor subclass whose calc_dist returns a numpy int64 CDF (one of 8
  precomputed tables per token): host time per token spent by the coder on the
  table (``_Tables.row`` + accept), and the whole encode of 256 tokens.

Bits are checked against the C oracle (static encode, bit-serial decode count)
on every run.  Prints one JSON line.  The reference's own speeds on the same
workload are measured in the build container by tools/ref_dropin_speed.py
(the reference cannot travel to the GPU box) and quoted in DESIGN.md.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from lac_amd import synth  # noqa: E402
from lac_amd.coder import AC, CDFPredictor, ProbPredictor, _Tables  # noqa: E402

V, PREC = 32000, 48


def static_table(seed=31):
    return synth.pmf_row(seed, 0, 0, V, "loguniform", 24).astype(np.uint64)


def draw(pmf, n, seed):
    cdf = np.cumsum(pmf.astype(np.float64))
    u = np.random.default_rng(seed).random(n) * cdf[-1]
    return np.minimum(np.searchsorted(cdf, u, side="right"), V - 1).astype(np.int64)


class NumpyCDF(ProbPredictor):
    """A model that emits a numpy int64 CDF per token (tables rotate with the token)."""

    def __init__(self, cdfs, i=0):
        super().__init__(V)
        self.cdfs, self.i = cdfs, i

    def calc_dist(self):
        self.dcache = self.cdfs[self.i % len(self.cdfs)]
        return self.dcache

    def accept(self, s):
        self.i += 1
        super().accept(s)

    def copy(self):
        return NumpyCDF(self.cdfs, self.i)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from oracle import oracle as coracle
    pmf = static_table()
    cdf = np.cumsum(pmf).astype(np.int64).tolist()          # a list of Python ints, as users build it
    syms = draw(pmf, a.n, 5).tolist()
    res = {"V": V, "prec": PREC, "n": a.n}

    # static encode: best of reps, a fresh coder each time (AC.to_bin makes one)
    ac = AC(CDFPredictor(cdf), PREC)
    R, L = ac.to_bin.encode(syms)                          # warm-up (library, device, allocation)
    t_enc = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        R, L = ac.to_bin.encode(syms)
        t_enc.append(time.perf_counter() - t0)
    want, wL, _ = coracle.encode(pmf, syms, PREC, static=True)
    data = R.to_bytes((L + 7) // 8, "big") if L else b""
    if L % 8:
        data = (R << (8 - L % 8)).to_bytes((L + 7) // 8, "big")
    res["encode_ok"] = bool(L == wL and data == want)
    res["encode_sym_per_s"] = a.n / min(t_enc)
    res["encode_ms"] = 1e3 * min(t_enc)
    bits = [int(b) for b in np.unpackbits(np.frombuffer(want, dtype=np.uint8))[:wL]]

    # static decode: run(bits, stop=0), the count the reference's bit-serial decoder emits
    t_dec = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        got = list(ac.from_bin.run(bits, stop=0))
        t_dec.append(time.perf_counter() - t0)
    ref_syms = coracle.decode_bitserial([pmf], want, wL, PREC, max_out=a.n + 1000)
    res["decode_ok"] = bool(got == ref_syms and got[:a.n] == syms)
    res["decode_sym_per_s"] = len(got) / min(t_dec)
    res["decode_ms"] = 1e3 * min(t_dec)
    res["decode_symbols"] = len(got)

    # numpy-CDF ProbPredictor: the coder's host time per token on the table
    rows = [synth.pmf_row(77, t, 0, V, "loguniform", 24).astype(np.int64) for t in range(8)]
    cdfs = [np.cumsum(r) for r in rows]
    p = NumpyCDF(cdfs)
    tab = _Tables(p, PREC)
    for _ in range(16):
        tab.row()
        tab.accept(0)
    t0 = time.perf_counter()
    k = 512
    for _ in range(k):
        tab.row()
        tab.accept(0)
    res["prob_host_ms_per_token"] = 1e3 * (time.perf_counter() - t0) / k
    toks = [int(draw(rows[t % 8].astype(np.uint64), 1, 100 + t)[0]) for t in range(256)]
    t0 = time.perf_counter()
    R2, L2 = AC(NumpyCDF(cdfs), PREC).to_bin.encode(toks)
    res["prob_encode_tok_per_s"] = len(toks) / (time.perf_counter() - t0)
    want2, wL2, _ = coracle.encode(np.stack([rows[t % 8] for t in range(256)]).astype(np.uint64), toks, PREC)
    data2 = (R2 << ((8 - L2 % 8) % 8)).to_bytes((L2 + 7) // 8, "big") if L2 else b""
    res["prob_encode_ok"] = bool(L2 == wL2 and data2 == want2)
    t0 = time.perf_counter()
    dec2 = list(AC(NumpyCDF(cdfs), PREC).from_bin.run(
        [int(b) for b in np.unpackbits(np.frombuffer(want2, dtype=np.uint8))[:wL2]], stop=0))
    res["prob_decode_tok_per_s"] = len(dec2) / (time.perf_counter() - t0)
    res["prob_decode_ok"] = bool(dec2[:256] == toks)
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            f.write(line + "\n")
    return 0 if all(v for k2, v in res.items() if k2.endswith("_ok")) else 1


if __name__ == "__main__":
    sys.exit(main())
