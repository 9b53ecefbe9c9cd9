#!/bin/bash
# Several bench.py configurations in one GPU session (each with its own limit).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/sweep
i=0
while IFS= read -r args; do
    [ -z "$args" ] && continue
    i=$((i+1))
    echo "== sweep $i: $args"
    timeout -k 10 600 python3 bench.py $args > "gpurun_out/sweep/$i.json" 2> "gpurun_out/sweep/$i.err"
    rc=$?
    echo "== rc=$rc"; tail -c 1500 "gpurun_out/sweep/$i.json"; echo
    if [ $rc -ne 0 ]; then tail -20 "gpurun_out/sweep/$i.err"; exit $rc; fi
done
