#!/bin/bash
# Round 5: k_decode_lean's step without per-step branches (the tests as sign bits and one
# exit test, branch-free renormalisation and window bits, the row i+2 prefetch clamped,
# the 1-padded end's target only past the stream's end, the stores out of line) vs the
# previous commit (tools/_probe/liblac_head.so): the whole GPU suite, c2 and 4 / 16 / 64
# streams (lean decode), the c3 headline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05ah}; mkdir -p $o
H=tools/_probe/liblac_head.so
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/gpu_tests.log 2>&1
rc=$?; tail -3 $o/gpu_tests.log; [ $rc -eq 0 ] || exit 3
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 5 --warmup 2 --decode-reps 3"
for r in 1 2 3; do
  timeout -k 10 200 $C2 > $o/c2_new$r.json 2> $o/c2_new$r.err || exit 3
  LAC_LIB=$H timeout -k 10 200 $C2 > $o/c2_head$r.json 2> $o/c2_head$r.err || exit 3
done
for s in 4 16 64; do
  B="python3 bench.py --cpu-baseline off --streams $s --tokens 1024 --steps 5 --warmup 2 --decode-reps 3"
  timeout -k 10 200 $B > $o/b${s}_new.json 2> $o/b${s}_new.err || exit 3
  LAC_LIB=$H timeout -k 10 200 $B > $o/b${s}_head.json 2> $o/b${s}_head.err || exit 3
done
timeout -k 10 300 python3 bench.py > $o/c3_headline.json 2> $o/c3_headline.err || exit 3
for f in $o/c2_*.json $o/b*_*.json $o/c3_headline.json; do python3 -c "
import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']; dd=p.get('decode',{})
print('$f'.split('/')[-1], 'enc %.3f M sym/s' % (d['value']/1e6), 'ms/step %.4f' % d['ms_per_step'], 'dec %.3f M' % (dd.get('symbols_per_s',0)/1e6), {k: round(v*1e3,3) for k,v in dd.get('kernel_ms_per_step_each',{}).items()}, 'oracle', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'))"; done
