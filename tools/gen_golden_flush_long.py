#!/usr/bin/env python3
"""Finish the decoder-flush golden vectors the 60 s limit of gen_golden_flush.py
cut off, and add fudged whole streams at the headline vocab (this container only).

    PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden_flush_long.py run  <k> [<k> ...]
    PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden_flush_long.py merge

The reference's A_from_bin.flush (arith_code.py:300-317) ranks every candidate
symbol the window straddles by overlap ratio, and each ratio recomputes the
V-entry fudged CDF in Python (:305-312 -> :86-93): O(V^2) per flush step at
V=32000 -- slow, not a loop.  `run k` re-runs job k with no time limit and
writes /tmp/flushlong/<k>.json; `merge` folds the finished jobs into
tests/golden/flush_cases.json (replacing the "timeout" records) and the new
generator cases into tests/golden/gen_cases.json.  Jobs (list with `jobs`):

* every flush_cases.json record whose exc is "timeout": same bits, same
  predictor, reference run(bits, stop=1) with no alarm;
* NEW_GEN: fudged V=32000 generator streams (encode goldens via
  gen_golden.gen_case, then the reference's run(bits, stop=1) on the whole
  stream).
"""
from __future__ import annotations

import json
import os
import sys
import time

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, "/root/reference")

import gen_golden  # noqa: E402
import gen_golden_flush as gf  # noqa: E402
from lac_amd import synth  # noqa: E402

GOLDEN = os.path.join(REPO, "tests", "golden")
OUT = "/tmp/flushlong"

# (name, seed, kind, exp_range, V, steps, prec, trace, decode): both fudge on
# every step (llama64 totals ~2^52+ against w <= 2^40; lu tables at prec 20)
NEW_GEN = [
    ("llama64_32000_p40", 25, "llama64", 0, 32000, 2, 40, True, False),
    ("lu32000_p20", 26, "loguniform", 24, 32000, 3, 20, True, False),
]


def _load(name):
    return json.load(open(os.path.join(GOLDEN, name)))


def jobs():
    fc = _load("flush_cases.json")["cases"]
    out = [("timeout", i) for i, c in enumerate(fc) if c["exc"] == "timeout"]
    out += [("new", j) for j in range(len(NEW_GEN))]
    return out


def _rows(g):
    return [[int(v) for v in synth.pmf_row(g["seed"], t, 0, g["V"], g["kind"], g["exp_range"])]
            for t in range(g["steps"])]


def run_job(k):
    kind, i = jobs()[k]
    t0 = time.time()
    if kind == "timeout":
        c = _load("flush_cases.json")["cases"][i]
        g = {x["name"]: x for x in _load("gen_cases.json")}[c["gen"]]
        rows = _rows(g)
        bits = gf.bits_of(c["bits"], c["nbits"])
        rec = gf.record(lambda: gen_golden.Replay(rows), c["prec"], bits, c["src"], 0)
        rec.update(gen=c["gen"], variant=c["variant"])
        res = {"kind": kind, "index": i, "record": rec}
    else:
        spec = NEW_GEN[i]
        g = gen_golden.gen_case(*spec)
        rows = _rows(g)
        bits = gf.bits_of(g["bytes"], g["L"])
        rec = gf.record(lambda: gen_golden.Replay(rows), g["prec"], bits, f"gen/{g['name']}", 0)
        rec.update(gen=g["name"], variant="whole")
        res = {"kind": kind, "gen_case": g, "record": rec}
    res["seconds"] = time.time() - t0
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, f"{k}.json"), "w") as f:
        json.dump(res, f)
    print(f"job {k} ({kind} {i}): {len(rec['out'])} symbols, exc {rec['exc']}, {res['seconds']:.0f}s", flush=True)


def merge():
    fpath, gpath = os.path.join(GOLDEN, "flush_cases.json"), os.path.join(GOLDEN, "gen_cases.json")
    fdoc, gen = json.load(open(fpath)), json.load(open(gpath))
    names = {g["name"] for g in gen}
    done = 0
    for k in range(len(jobs())):
        p = os.path.join(OUT, f"{k}.json")
        if not os.path.exists(p):
            print("job", k, "not finished")
            continue
        res = json.load(open(p))
        if res["kind"] == "timeout":
            old = fdoc["cases"][res["index"]]
            assert old["bits"] == res["record"]["bits"] and old["src"] == res["record"]["src"]
            # what the timed-out run yielded must be a prefix of the finished one
            assert res["record"]["out"][:len(old["out"])] == old["out"]
            fdoc["cases"][res["index"]] = res["record"]
        else:
            if res["gen_case"]["name"] not in names:
                gen.append(res["gen_case"])
                names.add(res["gen_case"]["name"])
            if not any(c["src"] == res["record"]["src"] for c in fdoc["cases"]):
                fdoc["cases"].append(res["record"])
        done += 1
    fdoc["generator"] = ("tools/gen_golden_flush.py + tools/gen_golden_flush_long.py (reference "
                         "arith_code.A_from_bin.run(bits, stop=1) and decode(R, L))")
    with open(fpath, "w") as f:
        json.dump(fdoc, f, separators=(",", ":"))
    with open(gpath, "w") as f:
        json.dump(gen, f, separators=(",", ":"))
    print(done, "jobs merged;", sum(c["exc"] == "timeout" for c in fdoc["cases"]), "timeouts left")


if __name__ == "__main__":
    if sys.argv[1] == "jobs":
        for k, j in enumerate(jobs()):
            print(k, j)
    elif sys.argv[1] == "run":
        for k in sys.argv[2:]:
            run_job(int(k))
    else:
        merge()
