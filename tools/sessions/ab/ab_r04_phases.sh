#!/bin/bash
# c2 lean decode phase split (probe build) + the product line.  gpurun -- bash tools/sessions/ab/ab_r04_phases.sh <outdir>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/${1:-phases}; mkdir -p $o
timeout -k 10 200 env LAC_LIB=tools/_probe/liblac_phases.so python3 tools/dec_phase_probe.py --kernel lean > $o/phases.json 2> $o/phases.err || { tail -20 $o/phases.err; exit 1; }
cat $o/phases.json
