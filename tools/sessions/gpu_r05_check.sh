#!/bin/bash
# Round 5, last check of the committed tree: the GPU suite, smoke and the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05check}; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/gpu_tests.log 2>&1
rc=$?; tail -3 $o/gpu_tests.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 3
tail -2 $o/smoke.log
timeout -k 10 300 python3 bench.py > $o/bench.json 2> $o/bench.err || exit 3
tail -1 $o/bench.json | cut -c1-400
