#!/bin/bash
# Round 6: where the wide u64 lean step's time goes: the c2 decode through tools/dec_phase_probe.py
# (kernel time per step) for u32 / u64 llama-scale rows, moving (one row per step) and static
# (one row, always L2-resident), and the moving u64 case without the helper waves.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06u}; mkdir -p $o
P="python3 tools/dec_phase_probe.py --tokens 4096"
timeout -k 10 200 $P > $o/u32_moving.json 2> $o/err.log || exit 3
timeout -k 10 200 $P --static > $o/u32_static.json 2>> $o/err.log || exit 3
timeout -k 10 200 $P --pmf-bits 64 > $o/u64_moving.json 2>> $o/err.log || exit 3
timeout -k 10 200 $P --pmf-bits 64 --static > $o/u64_static.json 2>> $o/err.log || exit 3
LAC_LIB=tools/_probe/liblac_nohelp.so timeout -k 10 200 $P --pmf-bits 64 > $o/u64_moving_nohelp.json 2>> $o/err.log || exit 3
LAC_LIB=tools/_probe/liblac_nohelp.so timeout -k 10 200 $P > $o/u32_moving_nohelp.json 2>> $o/err.log || exit 3
for f in $o/*.json; do echo "$(basename $f) $(cat $f | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["kernel_us_per_step"], d["round_trip"])')"; done
