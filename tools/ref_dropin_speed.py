#!/usr/bin/env python3
"""The REFERENCE's own speed on tools/dropin_bench.py's workload (this container
only: /root/reference never travels to the GPU box).

    PYTHONDONTWRITEBYTECODE=1 python tools/ref_dropin_speed.py > profiles/r04/ref_dropin_speed.json

Same static V=32000 table and symbols as dropin_bench.py: arith_code.AC(
CDFPredictor(cdf), 48).to_bin.encode(syms) and .from_bin.run(bits, stop=0)
(arith_code.py:76-110, 144-334); and the same numpy-CDF ProbPredictor subclass
(per token: calc_dist + the reference's minp + fudged_dist, :111-135).
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, "/root/reference")

import arith_code as ref  # noqa: E402  (the reference, read-only)
from dropin_bench import PREC, V, draw, static_table  # noqa: E402
from lac_amd import synth  # noqa: E402


class NumpyCDF(ref.ProbPredictor):
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


def main(n=10000):
    pmf = static_table()
    cdf = [int(x) for x in np.cumsum(pmf)]
    syms = draw(pmf, n, 5).tolist()
    ac = ref.AC(ref.CDFPredictor(cdf), PREC)
    t0 = time.perf_counter()
    R, L = ac.to_bin.encode(syms)
    t_enc = time.perf_counter() - t0
    bits = [(R >> (L - 1 - i)) & 1 for i in range(L)]
    t0 = time.perf_counter()
    dec = list(ac.from_bin.run(iter(bits), stop=0))
    t_dec = time.perf_counter() - t0
    assert dec[:n] == syms
    rows = [synth.pmf_row(77, t, 0, V, "loguniform", 24).astype(np.int64) for t in range(8)]
    cdfs = [[int(x) for x in np.cumsum(r)] for r in rows]   # exact ints: numpy int64 CDFs wrap (SURVEY finding 3)
    toks = [int(draw(rows[t % 8].astype(np.uint64), 1, 100 + t)[0]) for t in range(32)]
    t0 = time.perf_counter()
    ref.AC(NumpyCDF(cdfs), PREC).to_bin.encode(toks)
    t_prob = time.perf_counter() - t0
    print(json.dumps({"V": V, "prec": PREC, "n": n, "cores": 1,
                      "ref_static_encode_sym_per_s": n / t_enc, "ref_static_decode_sym_per_s": len(dec) / t_dec,
                      "ref_prob_ms_per_token": 1e3 * t_prob / len(toks),
                      "note": "reference arith_code.py run in the build container (Python 3.10, one core); "
                              "the ProbPredictor case uses exact-int list CDFs (a numpy int64 CDF wraps in "
                              "the reference's fudge test, SURVEY finding 3)"}))


if __name__ == "__main__":
    main()
