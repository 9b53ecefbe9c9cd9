#!/bin/bash
# Round 5: the (8 x 8) decode form of k_q1_stats with each row's cross-lane tail and
# stores deferred into the next row's second vector (LAC_Q1_TAIL_DEFER, product) vs at
# the row's end (tools/_probe/liblac_notail.so); logits / fuzz suites first,
# tools/q1_b2b.py at bf16 V = 32000 interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05ae}; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_logits.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/t.log 2>&1
rc=$?; tail -3 $o/t.log; [ $rc -eq 0 ] || exit 3
for r in 1 2 3; do
  timeout -k 10 200 python3 tools/q1_b2b.py --vocab 32000 --reps 20 > $o/b2b_new$r.json 2> $o/b2b_new$r.err || exit 3
  LAC_LIB=tools/_probe/liblac_notail.so timeout -k 10 200 python3 tools/q1_b2b.py --vocab 32000 --reps 20 > $o/b2b_base$r.json 2> $o/b2b_base$r.err || exit 3
done
for f in $o/b2b_*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); print('$f'.split('/')[-1], 'enc %.2f us/step' % (d['encode']['q1_stats_ms_per_launch']*1e3/16), 'dec %.2f us/step' % (d['decode']['q1_stats_ms_per_launch']*1e3/16), 'dec2 %.2f' % (d['decode2']['q1_stats_ms_per_launch']*1e3/16), 'q1dec %.2f' % d['decode']['q1_decode_us_per_step'])"; done
