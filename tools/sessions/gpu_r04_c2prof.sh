#!/bin/bash
# rocprofv3 kernel stats of the c2 decode (lean path) and the B=64 few-stream decode.
# gpurun -- bash tools/sessions/gpu_r04_c2prof.sh <outdir>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-c2prof}; mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/c2 -o run --output-format csv -- python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 3 --warmup 1 --decode-reps 3 > $o/c2.json 2> $o/c2.err || { tail -20 $o/c2.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/b64 -o run --output-format csv -- python3 bench.py --cpu-baseline off --streams 64 --tokens 512 --steps 3 --warmup 1 --decode-reps 3 > $o/b64.json 2> $o/b64.err || { tail -20 $o/b64.err; exit 1; }
find $o -type f -name '*kernel_trace.csv' -delete
python3 - "$o" <<'PY'
import csv, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/*/run_kernel_stats.csv")):
    print(f)
    for r in csv.DictReader(open(f)):
        if "anonymous namespace)::k_" in r["Name"]:
            print("  %-70s calls %6s avg %10.1f ns total %12.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]), float(r["TotalDurationNs"]) / 1e3))
PY
