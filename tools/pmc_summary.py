#!/usr/bin/env python3
"""Mean per-dispatch counter values per kernel from tools/sessions/pmc_passes.sh output.

    python3 tools/pmc_summary.py gpurun_out/<outdir> [kernel-substring]
FETCH_SIZE is also shown as bytes x2 (gfx950 wide-read correction, MI355X_MICROARCH.md)."""
import collections
import csv
import glob
import os
import re
import sys


def main(d, filt=""):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"]
                m = re.search(r"::(k_\w+)<([^>]*)>", k)
                name = f"{m.group(1)}<{m.group(2)[:40]}>" if m else k[:60]
                if filt and filt not in name:
                    continue
                vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for name, cs in sorted(vals.items()):
        print(name)
        for c, v in sorted(cs.items()):
            mean = sum(v) / len(v)
            extra = f"  ({mean * 2048 / 1e9:.3f} GB)" if c == "FETCH_SIZE" else ""
            print(f"   {c:28s} {mean:16.1f}  n={len(v)}{extra}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
