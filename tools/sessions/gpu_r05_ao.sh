#!/bin/bash
# Round 5: the post-suite dip of the headline bench -- the GPU suite, then the default
# bench at once, after 60 s idle, and with 200 warm jobs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05ao}; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/gpu_tests.log 2>&1 || exit 3
tail -1 $o/gpu_tests.log
timeout -k 10 300 python3 bench.py --cpu-baseline off > $o/after_suite.json 2> $o/after_suite.err || exit 3
timeout -k 10 300 python3 bench.py --cpu-baseline off --warmup 200 > $o/after_suite_w200.json 2> $o/after_suite_w200.err || exit 3
for i in 1 2 3 4 5 6; do sleep 10; echo idle $i; done
timeout -k 10 300 python3 bench.py --cpu-baseline off > $o/after_idle.json 2> $o/after_idle.err || exit 3
timeout -k 10 300 python3 bench.py --cpu-baseline off > $o/after_idle2.json 2> $o/after_idle2.err || exit 3
for f in after_suite after_suite_w200 after_idle after_idle2; do python3 -c "
import json; d=json.loads([l for l in open('$o/$f.json') if l.startswith('{')][-1]); r=d['roofline']
print('$f', '%.3f M sym/s' % (d['value']/1e6), 'kernel %.4f ms' % r['kernel_ms_per_launch'], 'frac', round(r['frac'],4))"; done
