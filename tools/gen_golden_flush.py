#!/usr/bin/env python3
"""Golden vectors for the decoder's flush: A_from_bin.run(bits, stop=1) and
decode(R, L) of the REFERENCE (arith_code.py:300-334), run here.

    PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden_flush.py

The decoder's flush (:300-317) picks, while [l, h] is not inside the received
window [lb, hb], the symbol of largest overlap ratio among those the window
straddles and emits it.  It raises on many inputs (SURVEY.md finding 5): the
records keep the symbols yielded before the exception and the exception itself
(type and its first argument, plus the symbol for 'unknown symbol').

Inputs (data only, output tests/golden/flush_cases.json):
* every small golden case (tests/golden/small_cases.json): its whole bitstream,
  two seeded prefixes of it and one copy with a flipped bit;
* uniform Predictor(n) streams (the floor mapping of AC()'s default, :64-74);
* the generator cases of tests/golden/gen_cases.json (V up to 32000): whole
  stream and one prefix.
A case the reference does not finish within the time limit is recorded as
"timeout" (its flush loops or runs O(V^2)); tests skip those.
"""
from __future__ import annotations

import json
import os
import random
import signal
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


class _Timeout(Exception):
    pass


def _alarm(*_):
    raise _Timeout()


def bits_of(hexbytes, L):
    data = bytes.fromhex(hexbytes)
    return [(data[i >> 3] >> (7 - (i & 7))) & 1 for i in range(L)]


def to_hex(bits):
    return bytes(ref.group_bits(iter(bits))).hex()


def outcome(gen, limit):
    """Drain a reference generator: (symbols yielded, exception record or None)."""
    out = []
    signal.signal(signal.SIGALRM, _alarm)
    signal.alarm(limit)
    try:
        for s in gen:
            out.append(int(s))
        exc = None
    except _Timeout:
        return out, "timeout"
    except AssertionError as e:
        exc = ["AssertionError", str(e.args[0])] + ([int(e.args[1])] if e.args and e.args[0] == "unknown symbol"
                                                   else [])
    except ZeroDivisionError as e:
        exc = ["ZeroDivisionError", str(e)]
    finally:
        signal.alarm(0)
    return out, exc


def record(pred_factory, prec, bits, src, limit, with_decode=False):
    out, exc = outcome(ref.AC(pred_factory(), prec).from_bin.run(iter(bits), stop=1), limit)
    rec = {"src": src, "prec": prec, "nbits": len(bits), "bits": to_hex(bits), "out": out, "exc": exc}
    if with_decode and exc != "timeout":
        R = int("".join(map(str, bits)) or "0", 2)
        dout, dexc = outcome(ref.AC(pred_factory(), prec).from_bin.decode(R, len(bits)), limit)
        rec["decode_out"], rec["decode_exc"] = dout, dexc
    # the bit-serial decoder fed bit by bit, then __call__(None) (:318-321)
    return rec


def main():
    rng = random.Random(20261017)
    small = json.load(open(os.path.join(GOLDEN, "small_cases.json")))
    cases = []
    for kind in ("static", "perstep"):
        for i, c in enumerate(small[kind]):
            bits = bits_of(c["bytes"], c["L"])
            mk = (lambda rows: (lambda: Replay(rows)))(c["rows"])
            cases.append(dict(record(mk, c["prec"], bits, f"small/{kind}/{i}", 20, with_decode=i % 5 == 0),
                              variant="whole"))
            for j in range(2):
                n = rng.randint(0, len(bits))
                cases.append(dict(record(mk, c["prec"], bits[:n], f"small/{kind}/{i}", 20), variant="prefix"))
            if bits:
                fb = list(bits)
                fb[rng.randrange(len(fb))] ^= 1
                cases.append(dict(record(mk, c["prec"], fb, f"small/{kind}/{i}", 20), variant="flipped"))
    print(len(cases), "small records", flush=True)
    for i in range(200):
        n = rng.randint(2, 12)
        prec = rng.randint(max(2, (n - 1).bit_length() + 1), 18)
        syms = [rng.randrange(n) for _ in range(rng.randint(0, 14))]
        bits = list(ref.AC(ref.Predictor(n), prec).to_bin.bits(syms))
        mk = (lambda n: (lambda: ref.Predictor(n)))(n)
        variant = ("whole", "prefix", "flipped")[i % 3]
        if variant == "prefix":
            bits = bits[:rng.randint(0, len(bits))]
        elif variant == "flipped" and bits:
            bits[rng.randrange(len(bits))] ^= 1
        rec = record(mk, prec, bits, f"uniform/{i}", 20, with_decode=i % 4 == 0)
        rec.update(uniform=n, syms=syms, variant=variant)
        cases.append(rec)
    print(len(cases), "records with uniform", flush=True)
    gen = json.load(open(os.path.join(GOLDEN, "gen_cases.json")))
    for c in gen:
        rows = [synth.pmf_row(c["seed"], t, 0, c["V"], c["kind"], c["exp_range"]) for t in range(c["steps"])]
        rows = [[int(v) for v in r] for r in rows]
        bits = bits_of(c["bytes"], c["L"])
        mk = (lambda rows: (lambda: Replay(rows)))(rows)
        for variant, bb in (("whole", bits), ("prefix", bits[:rng.randint(0, len(bits))])):
            rec = record(mk, c["prec"], bb, f"gen/{c['name']}", 60)
            rec.update(gen=c["name"], variant=variant)
            cases.append(rec)
            print(f"  {c['name']} {variant}: {len(rec['out'])} symbols, exc {rec['exc']}", flush=True)
    with open(os.path.join(GOLDEN, "flush_cases.json"), "w") as f:
        json.dump({"generator": "tools/gen_golden_flush.py (reference arith_code.A_from_bin.run(bits, stop=1) "
                                "and decode(R, L))", "cases": cases}, f, separators=(",", ":"))
    n_exc = sum(1 for c in cases if c["exc"] not in (None, "timeout"))
    n_to = sum(1 for c in cases if c["exc"] == "timeout")
    print(len(cases), "cases,", n_exc, "raise,", n_to, "timeouts")


if __name__ == "__main__":
    main()
