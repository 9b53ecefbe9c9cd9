#!/usr/bin/env python3
"""Golden vectors for predictors with their own mapping, and for debug_log,
from the REFERENCE coder (arith_code.py:156-334) run here.

    PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden_custom.py

Predictors: tests/custom_predictors.py built over the reference's Predictor /
CDFPredictor.  Recorded per case: A_to_bin bits and debug_log, and what
A_from_bin.run(bits, stop=1) and run(bits, stop=0) yield (with the exception,
if any).  Plus debug_log of a few CDFPredictor (table) encodes.
Output tests/golden/custom_cases.json (data only).
"""
from __future__ import annotations

import itertools
import json
import os
import random
import signal
import sys

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, "/root/reference")

import arith_code as ref  # noqa: E402  (the reference, read-only)
import custom_predictors  # noqa: E402

GOLDEN = os.path.join(REPO, "tests", "golden")
Fixed, FloorCDF, Counting = custom_predictors.make(ref.Predictor, ref.CDFPredictor)


class _Timeout(BaseException):
    pass


def _alarm(*_):
    raise _Timeout()


def outcome(gen, limit=10):
    """(symbols yielded, [exception type, first argument] or None, or "timeout")."""
    out = []
    signal.signal(signal.SIGALRM, _alarm)
    signal.alarm(limit)
    try:
        for v in gen:
            out.append(int(v))
    except _Timeout:
        return out[:64], "timeout"
    except Exception as e:                            # noqa: BLE001 -- recorded, whatever it is
        return out, [type(e).__name__, str(e.args[0]) if e.args else ""]
    finally:
        signal.alarm(0)
    return out, None


def case(kind, params, prec, syms):
    mk = lambda: custom_predictors.build(kind, Fixed, FloorCDF, Counting, params)   # noqa: E731
    enc = ref.AC(mk(), prec).to_bin
    enc.debug_log = ["start"]                         # the reference logs only into a truthy list
    bits, exc = outcome(enc.bits(syms))
    if exc is not None:
        return {"kind": kind, "params": params, "prec": prec, "syms": syms, "encode_exc": exc}
    log = [list(x) if isinstance(x, tuple) else x for x in enc.debug_log]
    rec = {"kind": kind, "params": params, "prec": prec, "syms": syms, "bits": "".join(map(str, bits)),
           "debug_log": log}
    rec["stop1"] = outcome(ref.AC(mk(), prec).from_bin.run(iter(bits), stop=1))
    rec["stop0"] = outcome(ref.AC(mk(), prec).from_bin.run(iter(bits), stop=0))
    return rec


def main():
    rng = random.Random(20261018)
    cases = []
    for i in range(60):
        kind = ("fixed", "floorcdf", "counting")[i % 3]
        if kind == "fixed":
            n = rng.randint(2, 6)
            edges = list(itertools.accumulate(rng.randint(1, 4) for _ in range(n)))
            prec = rng.randint(max(3, edges[-1].bit_length() + 1), 20)
            params = edges
        elif kind == "floorcdf":
            n = rng.randint(2, 9)
            params = list(itertools.accumulate(rng.choice([1, 2, 5, 30, 400]) for _ in range(n)))
            prec = rng.randint(max(4, n.bit_length() + 2), 24)
        else:
            n = rng.randint(2, 9)
            params = n
            prec = rng.randint(max(4, n.bit_length() + 2), 32)
        syms = [rng.randrange(n) for _ in range(rng.randint(0, 25))]
        cases.append(case(kind, params, prec, syms))
    tables = []
    for i in range(8):
        n = rng.randint(2, 8)
        cdf = list(itertools.accumulate(rng.choice([1, 3, 50, 700]) for _ in range(n)))
        prec = rng.randint(max(4, n.bit_length() + 2), 30)
        syms = [rng.randrange(n) for _ in range(rng.randint(1, 20))]
        enc = ref.AC(ref.CDFPredictor(cdf), prec).to_bin
        enc.debug_log = ["start"]
        bits = list(enc.bits(syms))
        tables.append({"cdf": cdf, "prec": prec, "syms": syms, "bits": "".join(map(str, bits)),
                       "debug_log": [list(x) if isinstance(x, tuple) else x for x in enc.debug_log]})
    with open(os.path.join(GOLDEN, "custom_cases.json"), "w") as f:
        json.dump({"generator": "tools/gen_golden_custom.py (reference arith_code AC over tests/custom_predictors)",
                   "cases": cases, "table_logs": tables}, f, separators=(",", ":"))
    print(len(cases), "cases;", sum(1 for c in cases if "encode_exc" in c), "encode raises;",
          sum(1 for c in cases if c.get("stop1", [0, None])[1] not in (None,)), "stop1 raises")


if __name__ == "__main__":
    main()
