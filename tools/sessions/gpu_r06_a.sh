#!/bin/bash
# Round 6, first session: attribute the drop-in static decode (AC(CDFPredictor).from_bin.run,
# VERDICT r5 item 1) -- kernel trace + HIP API trace of tools/dropin_bench.py -- and the
# round-start c2 u32 / u64 lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06a}; mkdir -p $o
timeout -k 10 300 python3 tools/dropin_bench.py --out $o/dropin.json > $o/dropin.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats -d $o/trace -o run --output-format csv -- python3 tools/dropin_bench.py --reps 1 > $o/dropin_trace.log 2>&1 || exit 3
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 5 --warmup 2 --decode-reps 3"
timeout -k 10 200 $C2 > $o/c2.json 2> $o/c2.err || exit 3
timeout -k 10 200 $C2 --pmf-bits 64 > $o/c2_u64.json 2> $o/c2_u64.err || exit 3
cat $o/dropin.json
ls $o/trace
