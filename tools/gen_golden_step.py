#!/usr/bin/env python3
"""Golden vectors for bit-serial decoding: A_from_bin.step(bit) of the REFERENCE
(arith_code.py:291-298) run here over the bits of existing golden cases.

    PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden_step.py

For each case it records, per input bit, how many symbols the reference's
step(bit) yields (the symbols themselves are the case's syms followed by its
decoded_extra).  Inputs are the cases already in tests/golden (rows / syms /
bytes / L); output tests/golden/step_cases.json (data only).
"""
from __future__ import annotations

import json
import os
import sys

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, "/root/reference")

import arith_code as ref  # noqa: E402  (the reference, read-only)
from gen_golden import Replay  # noqa: E402
from lac_amd import synth  # noqa: E402

GOLDEN = os.path.join(REPO, "tests", "golden")


def bits_of(hexbytes, L):
    data = bytes.fromhex(hexbytes)
    return [(data[i >> 3] >> (7 - (i & 7))) & 1 for i in range(L)]


def step_counts(rows, prec, bits):
    dec = ref.AC(Replay(rows), prec).from_bin
    counts, syms = [], []
    for b in bits:
        out = list(dec.step(b))
        counts.append(len(out))
        syms.extend(out)
    return counts, syms


def main():
    small = json.load(open(os.path.join(GOLDEN, "small_cases.json")))
    gen = json.load(open(os.path.join(GOLDEN, "gen_cases.json")))
    cases = []
    for kind in ("static", "perstep"):
        for i, c in enumerate(small[kind][:40]):
            if c["L"] == 0:
                continue
            counts, syms = step_counts(c["rows"], c["prec"], bits_of(c["bytes"], c["L"]))
            cases.append({"src": f"small/{kind}/{i}", "rows": c["rows"], "prec": c["prec"], "L": c["L"],
                          "bytes": c["bytes"], "counts": counts, "syms": syms})
    gcases = gen["cases"] if isinstance(gen, dict) else gen
    for c in gcases:
        if c["V"] > 1000 or c["kind"] == "llama64":
            continue
        rows = [synth.pmf_row(c["seed"], t, 0, c["V"], c["kind"], c["exp_range"]) for t in range(c["steps"])]
        counts, syms = step_counts(rows, c["prec"], bits_of(c["bytes"], c["L"]))
        cases.append({"src": f"gen/{c['name']}", "gen": c["name"], "prec": c["prec"], "L": c["L"],
                      "bytes": c["bytes"], "counts": counts, "syms": syms})
        print(f"  {c['name']}: {len(syms)} symbols over {c['L']} bits", flush=True)
    with open(os.path.join(GOLDEN, "step_cases.json"), "w") as f:
        json.dump({"generator": "tools/gen_golden_step.py (reference arith_code.A_from_bin.step)",
                   "cases": cases}, f)
    print(len(cases), "cases")


if __name__ == "__main__":
    main()
