#!/bin/bash
# Round 5: host-side timeline of the gather (LAC_GATHER_TRACE) over repeated runs,
# to find the run-to-run stalls of the batched form.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05f}; mkdir -p $o
for r in 1 2 3 4; do
  LAC_GATHER_TRACE=$o/trace$r.jsonl timeout -k 10 200 python3 bench.py --gather --steps 40 --warmup 5 --cpu-baseline off > $o/gather$r.json 2> $o/gather$r.err || exit 3
done
timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --cpu-baseline off > $o/plain1.json 2> $o/plain1.err || exit 3
python3 tools/sessions/ab/summ.py $o
