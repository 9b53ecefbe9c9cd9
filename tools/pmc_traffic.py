#!/usr/bin/env python3
"""Per-launch HBM read traffic from a rocprofv3 --pmc FETCH_SIZE run.

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc -o run --output-format csv \
        -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline off
    python tools/pmc_traffic.py gpurun_out/pmc [--input pmf|logits-bf16|logits-f32] [--vocab V --tokens T]
        (adds / replaces this configuration's entry in profiles/pmc_traffic.json)

FETCH_SIZE is reported in KiB.  On gfx950 it reads exactly half of the bytes of
a wide (16 B/lane) coalesced streaming read (MI355X_MICROARCH.md, HBM section),
so bytes = FETCH_SIZE * 1024 * 2 for the row-streaming kernels, whose loads are
all global_load_dwordx4.  The median over dispatches of each kernel is kept.
"""
import csv
import glob
import json
import os
import statistics
import sys

STREAMING = ("k_encode_fused", "k_row_stats", "k_decode_step", "k_decode_wave_fine", "k_decode_wave",
             "k_q1_stats", "k_q1_stats_dec", "k_dec_stats")


def _q1_decode_form(name):
    """True when a k_q1_stats* kernel name is the decode form (its DEC template argument)."""
    import re
    m = re.search(r"::(k_q1_stats(?:_wide|_rl)?)<([^>]*)>", name)
    if not m:
        return False
    args = [x.strip() for x in m.group(2).split(",")]
    pos = {"k_q1_stats": 3, "k_q1_stats_wide": 2, "k_q1_stats_rl": 1}[m.group(1)]
    return len(args) > pos and args[pos] == "true"


def short(name):
    if "::k_q1_stats" in name:        # the row stats (incl. register + LDS-slot / 8-wave forms), by direction
        return "k_q1_stats_dec" if _q1_decode_form(name) else "k_q1_stats"
    for k in STREAMING + ("k_encode", "k_finish", "k_q1_decode", "k_decode_seq"):
        if f"::{k}<" in name or f"::{k}(" in name:
            return k
    return None


def main(d, vocab=32000, streams=4096, tokens=16, pmf_bits=32, inp="pmf", out_path=None):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        sys.exit(f"no counter_collection.csv under {d}")
    per = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != "FETCH_SIZE":
                    continue
                k = short(row.get("Kernel_Name", ""))
                if k:
                    per.setdefault(k, []).append(float(row["Counter_Value"]))
    ent = {"vocab": vocab, "streams": streams, "tokens": tokens, "pmf_bits": pmf_bits, "input": inp,
           "counter": "FETCH_SIZE (KiB), x1024 x2 gfx950 wide-read correction", "bytes_per_launch": {},
           "raw_fetch_kib_median": {}, "dispatches": {}}
    for k, v in per.items():
        # a row-group launch is followed by a repair launch gated on its abort word, which
        # exits at once (a few KiB): those dispatches are not the kernel's traffic
        big = [x for x in v if x >= 0.01 * max(v)]
        v = big or v
        med = statistics.median(v)
        ent["raw_fetch_kib_median"][k] = med
        ent["dispatches"][k] = len(v)
        ent["bytes_per_launch"][k] = med * 1024 * (2 if k in STREAMING else 1)
    doc = {"entries": []}
    if out_path and os.path.exists(out_path):
        with open(out_path) as fh:
            old = json.load(fh)
        doc["entries"] = [e for e in old.get("entries", [])
                          if any(e.get(k) != ent[k] for k in ("vocab", "streams", "tokens", "pmf_bits", "input"))]
    doc["entries"].append(ent)
    text = json.dumps(doc, indent=1)
    if out_path:
        with open(out_path, "w") as fh:
            fh.write(text + "\n")
    print(text)


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("dir", nargs="?", default="gpurun_out/pmc")
    ap.add_argument("--vocab", type=int, default=32000)
    ap.add_argument("--streams", type=int, default=4096)
    ap.add_argument("--tokens", type=int, default=16)
    ap.add_argument("--pmf-bits", type=int, default=32)
    ap.add_argument("--input", default="pmf")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles",
                                                  "pmc_traffic.json"))
    a = ap.parse_args()
    main(a.dir, a.vocab, a.streams, a.tokens, a.pmf_bits, a.input, a.out)
