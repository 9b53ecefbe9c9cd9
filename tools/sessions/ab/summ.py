#!/usr/bin/env python3
"""Summarise an A/B directory of bench JSON lines: value, roofline frac and decode rate per file."""
import glob
import json
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    try:
        line = [l for l in open(f) if l.startswith("{")][-1]
        j = json.loads(line)
    except (IndexError, ValueError):
        print(f"{os.path.basename(f):28s} (no result)")
        continue
    r = j["roofline"]
    dec = j["parity"]["decode"]
    print(f"{os.path.basename(f):28s} {j['value'] / 1e6:8.2f} M/s  {r['kernel']:16s} {r['kernel_ms_per_launch']:.4f} ms "
          f"{r['achieved']:7.0f} GB/s ({r['frac'] * 100:4.1f} %)  dec {dec['symbols_per_s'] / 1e6:6.2f} M/s  "
          f"rt={j['parity']['round_trip_all_streams']}")
    each = dec.get("kernel_ms_per_step_each")
    if each:
        print(" " * 30 + "decode ms/step: " + ", ".join(f"{k} {v * 1e3:.1f} us" for k, v in each.items()))
