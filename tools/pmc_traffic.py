#!/usr/bin/env python3
"""Per-launch HBM read traffic from a rocprofv3 --pmc FETCH_SIZE run.

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc -o run --output-format csv \
        -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline off
    python tools/pmc_traffic.py gpurun_out/pmc > profiles/pmc_traffic.json

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

STREAMING = ("k_encode_fused", "k_row_stats", "k_decode_step")


def short(name):
    for k in STREAMING + ("k_encode", "k_finish"):
        if f"::{k}<" in name or f"::{k}(" in name:
            return k
    return None


def main(d, vocab=32000, streams=4096, tokens=16, pmf_bits=32):
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
    out = {"vocab": vocab, "streams": streams, "tokens": tokens, "pmf_bits": pmf_bits,
           "counter": "FETCH_SIZE (KiB), x1024 x2 gfx950 wide-read correction", "bytes_per_launch": {},
           "raw_fetch_kib_median": {}, "dispatches": {}}
    for k, v in per.items():
        med = statistics.median(v)
        out["raw_fetch_kib_median"][k] = med
        out["dispatches"][k] = len(v)
        out["bytes_per_launch"][k] = med * 1024 * (2 if k in STREAMING else 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
