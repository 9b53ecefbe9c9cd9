#!/usr/bin/env python3
"""What runs between consecutive encode launches in a rocprofv3 --kernel-trace CSV:
per gap its length and the kernels that started inside it (name, start after the
previous encode's end, duration, hardware queue).  Used to attribute the gather's
cost per job (profiles/r05/gather/).

    python3 tools/gather_gaps.py <dir with *kernel_trace.csv> [--kernel k_encode_fused] [--skip 3]
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="k_encode_fused")
    ap.add_argument("--skip", type=int, default=3, help="encode launches to skip (warmup)")
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    enc = [i for i, r in enumerate(rows) if a.kernel in r["Kernel_Name"]]
    gaps, durs = [], []
    for x, y in zip(enc[a.skip:-1], enc[a.skip + 1:]):
        ra, rb = rows[x], rows[y]
        end = int(ra["End_Timestamp"])
        durs.append((end - int(ra["Start_Timestamp"])) / 1e3)
        gaps.append((int(rb["Start_Timestamp"]) - end) / 1e3)
        inside = ["%s +%.1f d%.1f q%s" % (r["Kernel_Name"][:32], (int(r["Start_Timestamp"]) - end) / 1e3,
                                          (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, r["Queue_Id"])
                  for r in rows[x + 1:y]]
        print("encode %.1f us, gap %.1f us  %s" % (durs[-1], gaps[-1], "; ".join(inside)))
    print("mean: encode %.1f us, gap %.1f us over %d gaps" % (sum(durs) / len(durs), sum(gaps) / len(gaps), len(gaps)))


if __name__ == "__main__":
    main()
