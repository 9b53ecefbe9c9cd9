#!/bin/bash
# Round 5: full GPU suite + smoke + headline bench (+ bf16 logits line) on the split
# translation units, and the rocprofv3 kernel stats of the headline command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05full}; mkdir -p $o
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/gpu_tests.log 2>&1
rc=$?; tail -3 $o/gpu_tests.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 3
cat $o/smoke.log | tail -1
timeout -k 10 300 python3 bench.py > $o/bench.json 2> $o/bench.err || exit 3
timeout -k 10 300 python3 bench.py --input logits-bf16 --cpu-baseline off > $o/bench_bf16.json 2> $o/bench_bf16.err || exit 3
python3 tools/sessions/ab/summ.py $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run --output-format csv -- python3 bench.py --cpu-baseline off > $o/prof.log 2>&1 || exit 3
