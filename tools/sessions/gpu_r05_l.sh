#!/bin/bash
# Round 5: c2 encode phase breakdown (probe build), c2 bench lines, and the headline A/B
# split-TU library vs the pre-split one (same box, interleaved).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05l}; mkdir -p $o
LAC_LIB=tools/_probe/liblac_encphases.so timeout -k 10 200 python3 tools/enc_phase_probe.py > $o/enc_phases.json 2> $o/enc_phases.err || exit 3
cat $o/enc_phases.json
timeout -k 10 200 python3 tools/enc_phase_probe.py > $o/enc_plain.json 2> $o/enc_plain.err || exit 3
cat $o/enc_plain.json
timeout -k 10 300 python3 bench.py --streams 1 --tokens 4096 --steps 3 --warmup 1 --cpu-baseline off > $o/c2.json 2> $o/c2.err || exit 3
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --cpu-baseline off --steps 40 --warmup 5 > $o/split$r.json 2> $o/split$r.err || exit 3
  LAC_LIB=tools/_probe/liblac_presplit.so timeout -k 10 300 python3 bench.py --cpu-baseline off --steps 40 --warmup 5 > $o/presplit$r.json 2> $o/presplit$r.err || exit 3
done
python3 tools/sessions/ab/summ.py $o
