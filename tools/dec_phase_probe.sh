#!/bin/bash
# Build the phase-probe variant of liblac (k_decode_seq with s_memtime marks) and run
# tools/dec_phase_probe.py on the c2 workload.  gpurun -- bash tools/dec_phase_probe.sh
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/${1:-phases}; mkdir -p $o
timeout -k 10 300 env LAC_LIB=tools/_probe/liblac_phases.so python3 tools/dec_phase_probe.py > $o/phases.json 2> $o/phases.err
cat $o/phases.json
