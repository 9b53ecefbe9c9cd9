#!/usr/bin/env python3
"""Golden vectors for the caller-side quantiser: the REFERENCE's Llama_AC
(llama_compress.py:14-61) driven by a fake llm (tests/fake_llm.py), run here.

    PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden_llama.py

llama_compress imports llama_cpp only inside r() (:5), so its Llama_AC runs with
any object of llama_cpp.Llama's duck type.  For each configuration the fake llm
yields seeded float32 logits that depend on the context window; n_ctx is small
so the sliding window (:33-36) wraps several times.  Recorded per step: sha256
of the float32 logits, sha256 of the int64 CDF calc_dist returns (:24-30), the
minp property (:43-45), and the full CDFs of the first steps; then the bits that
A_to_bin gives on those CDFs as exact Python ints (a Replay CDFPredictor, the
parity contract, SURVEY.md finding 3) and, for the record, the bits of the
reference's Llama_AC coded as it is (numpy int64 arithmetic, which wraps).
The exact-int coder reads each row's minp from the reference's own Llama_AC.minp
(llama_compress.py:43-45), zeros included: peaky rows (``scale`` 12) whose float
cumsum absorbs small entries have zero CDF steps, minp 0, and then always take
fudged_dist (arith_code.py:84).  A "refuse" case (HeadLlama: every positive entry
>= 2^12 next to zero steps) records rows where that decision differs from the one
the table's smallest positive entry gives at some interval width: the reference
codes them, this build refuses them (lac_amd.coder.fudge_decisions_agree).
Output tests/golden/llama_cases.json (data only).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, "/root/reference")

import numpy as np  # noqa: E402

import arith_code as ref  # noqa: E402  (the reference, read-only)
import llama_compress as lc  # noqa: E402  (the reference, read-only)
from fake_llm import FakeLlama, HeadLlama  # noqa: E402

GOLDEN = os.path.join(REPO, "tests", "golden")
CONFIGS = [  # (name, vocab, n_ctx, seed, tokens, prec, full_cdf_steps, scale)
    ("v1000_ctx12", 1000, 12, 101, 40, 48, 2, 3.0),
    ("v257_ctx8", 257, 8, 202, 30, 48, 5, 3.0),
    ("v32000_ctx6", 32000, 6, 303, 14, 48, 0, 3.0),
    ("v1000_peaky_ctx10", 1000, 10, 404, 36, 48, 2, 12.0),      # zero CDF steps: minp 0
    ("v32000_peaky_ctx6", 32000, 6, 505, 12, 48, 0, 12.0),
]
# rows whose positive entries are all >= 2^12: [2^60-ish, big, big, 0, 0, ...]
REFUSE = ("v1000_refuse", 1000, 6, [[50.0, 45.0, 40.0], [48.0, 44.0, 41.0, 39.0]], 10.0, 5, 48)


class ReplayMinp(ref.CDFPredictor):
    """The reference's CDFPredictor replaying recorded rows (Python ints) with a
    recorded minp per row -- the reference Llama_AC's own, zeros included."""

    def __init__(self, rows, minps):
        self.rows, self.minps = rows, minps
        self.i = 0
        self._load()

    def _load(self):
        k = min(self.i, len(self.rows) - 1)
        acc, cdf = 0, []
        for v in self.rows[k]:
            acc += int(v)
            cdf.append(acc)
        self.dist = cdf
        self.minp = int(self.minps[k])

    def accept(self, symbol):
        self.i += 1
        self._load()

    def copy(self):
        return ReplayMinp(self.rows, self.minps)


def sha(b):
    return hashlib.sha256(b).hexdigest()


def record(llm, toks, nfull):
    """Drive the reference's Llama_AC over toks; per step the logits, CDF, minp and window."""
    p = lc.Llama_AC(llm)
    steps, rows, minps = [], [], []
    for i, t in enumerate(toks):
        logits = np.asarray(llm._scores[-1], dtype=np.float32)
        cdf = p.dist                                   # calc_dist, cached until accept
        rec = {"logits_sha256": sha(logits.tobytes()), "cdf_sha256": sha(np.asarray(cdf, dtype="<i8").tobytes()),
               "minp": int(p.minp), "window": len(p.past)}
        if i < nfull:
            rec["cdf"] = [int(x) for x in cdf]
        steps.append(rec)
        c = [int(x) for x in cdf]
        rows.append([c[0]] + [c[j + 1] - c[j] for j in range(len(c) - 1)])
        minps.append(int(p.minp))
        p.accept(t)
    return steps, rows, minps


def exact_bits(rows, minps, toks, prec):
    bits = list(ref.AC(ReplayMinp(rows, minps), prec).to_bin.bits(toks))
    return len(bits), bytes(ref.group_bits(iter(bits))).hex()


def run(name, V, n_ctx, seed, T, prec, nfull, scale):
    rng = np.random.default_rng(seed)
    toks = [int(t) for t in rng.integers(0, V, T)]
    steps, rows, minps = record(FakeLlama(V, n_ctx, seed, scale=scale), toks, nfull)
    L, data = exact_bits(rows, minps, toks, prec)
    as_is = list(ref.AC(lc.Llama_AC(FakeLlama(V, n_ctx, seed, scale=scale)), prec).to_bin.bits(toks))
    zero_rows = sum(1 for r in rows if 0 in r)
    print(f"  {name}: {L} bits exact-int, {len(as_is)} bits as-is, {zero_rows}/{T} rows with zero steps",
          flush=True)
    return {"name": name, "vocab": V, "n_ctx": n_ctx, "seed": seed, "scale": scale, "prec": prec, "tokens": toks,
            "steps": steps, "zero_step_rows": zero_rows, "exact_L": L, "exact_bytes": data,
            "as_is_L": len(as_is), "as_is_bytes": bytes(ref.group_bits(iter(as_is))).hex()}


def run_refuse(name, V, n_ctx, heads, floor, T, prec):
    """Rows the reference fudges (minp 0) where the smallest positive entry (>= 2^12)
    would leave some widths unfudged: recorded with the reference's bits, and which
    step the build must refuse at (the first such row)."""
    toks = [int(t) for t in np.random.default_rng(606).integers(0, V, T)]
    steps, rows, minps = record(HeadLlama(V, n_ctx, heads, floor), toks, 1)
    L, data = exact_bits(rows, minps, toks, prec)
    lo_w, hi_w = (1 << (prec - 1)) + 1, 1 << prec
    first = None
    for k, r in enumerate(rows):
        T_, mp = sum(r), min(v for v in r if v > 0)
        fud_ref = [T_ > w * minps[k] for w in (lo_w, hi_w)]
        fud_pos = [T_ > w * mp for w in (lo_w, hi_w)]
        if fud_ref != fud_pos and first is None:
            first = k
    assert first is not None, "no refusal row"
    print(f"  {name}: {L} bits exact-int, build refuses at step {first}", flush=True)
    return {"name": name, "vocab": V, "n_ctx": n_ctx, "heads": heads, "floor": floor, "prec": prec, "tokens": toks,
            "steps": steps, "min_positive": [min(v for v in r if v > 0) for r in rows], "exact_L": L,
            "exact_bytes": data, "refuse_at_step": first}


def main():
    cases = [run(*c) for c in CONFIGS]
    refuse = [run_refuse(*REFUSE)]
    with open(os.path.join(GOLDEN, "llama_cases.json"), "w") as f:
        json.dump({"generator": "tools/gen_golden_llama.py (reference llama_compress.Llama_AC + fake llm)",
                   "cases": cases, "refuse": refuse}, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
