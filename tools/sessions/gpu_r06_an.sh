#!/bin/bash
# Round 6: where V = 65536 u64 rows' one-stream decode time goes (2.6 us per step against
# 1.28 at V = 32000): the decode probe on moving and static rows, u64 and u32, 2048 steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06an}; mkdir -p $o
P="python3 tools/dec_phase_probe.py --tokens 2048 --vocab 65536"
timeout -k 10 200 $P --pmf-bits 64 > $o/u64_moving.json 2> $o/err.log || exit 3
timeout -k 10 200 $P --pmf-bits 64 --static > $o/u64_static.json 2>> $o/err.log || exit 3
timeout -k 10 200 $P --pmf-bits 64 --scale-bits 40 > $o/u64_s40_moving.json 2>> $o/err.log || exit 3
timeout -k 10 200 $P > $o/u32_moving.json 2>> $o/err.log || exit 3
for f in $o/*.json; do echo "$(basename $f) $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["kernel_us_per_step"], d["round_trip"])' $f)"; done
