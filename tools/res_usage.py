#!/usr/bin/env python3
"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks: VGPRs / spills per kernel.
   python3 tools/res_usage.py <stderr file> [substring]"""
import re
import subprocess
import sys

text = open(sys.argv[1]).read().split("\n")
want = sys.argv[2] if len(sys.argv) > 2 else ""
cur, info = None, {}
for line in text:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        info[cur] = {}
        continue
    for key in ("VGPRs", "AGPRs", "VGPRs Spill", "SGPRs Spill", "LDS Size \\[bytes/block\\]", "Occupancy \\[waves/SIMD\\]"):
        m = re.search(key + r":\s*(\d+)", line)
        if m and cur:
            info[cur][key.split(" \\[")[0]] = int(m.group(1))
for f, d in info.items():
    name = subprocess.run(["c++filt", f], capture_output=True, text=True).stdout.strip()
    if want not in name:
        continue
    name = name.replace("void (anonymous namespace)::", "").split(">(")[0] + ">"
    print(f"{name:80s} " + " ".join(f"{k}={v}" for k, v in d.items()))
