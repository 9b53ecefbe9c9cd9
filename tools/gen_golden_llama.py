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
from fake_llm import FakeLlama  # noqa: E402
from gen_golden import Replay  # noqa: E402

GOLDEN = os.path.join(REPO, "tests", "golden")
CONFIGS = [  # (name, vocab, n_ctx, seed, tokens, prec, full_cdf_steps)
    ("v1000_ctx12", 1000, 12, 101, 40, 48, 2),
    ("v257_ctx8", 257, 8, 202, 30, 48, 5),
    ("v32000_ctx6", 32000, 6, 303, 14, 48, 0),
]


def sha(b):
    return hashlib.sha256(b).hexdigest()


def run(name, V, n_ctx, seed, T, prec, nfull):
    rng = np.random.default_rng(seed)
    toks = [int(t) for t in rng.integers(0, V, T)]
    llm = FakeLlama(V, n_ctx, seed)
    p = lc.Llama_AC(llm)
    steps, rows = [], []
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
        p.accept(t)
    exact = ref.AC(Replay(rows), prec).to_bin
    bits = list(exact.bits(toks))
    as_is = list(ref.AC(lc.Llama_AC(FakeLlama(V, n_ctx, seed)), prec).to_bin.bits(toks))
    print(f"  {name}: {len(bits)} bits exact-int, {len(as_is)} bits as-is", flush=True)
    return {"name": name, "vocab": V, "n_ctx": n_ctx, "seed": seed, "prec": prec, "tokens": toks, "steps": steps,
            "exact_L": len(bits), "exact_bytes": bytes(ref.group_bits(iter(bits))).hex(),
            "as_is_L": len(as_is), "as_is_bytes": bytes(ref.group_bits(iter(as_is))).hex()}


def main():
    cases = [run(*c) for c in CONFIGS]
    with open(os.path.join(GOLDEN, "llama_cases.json"), "w") as f:
        json.dump({"generator": "tools/gen_golden_llama.py (reference llama_compress.Llama_AC + fake llm)",
                   "cases": cases}, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
