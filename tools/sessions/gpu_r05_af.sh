#!/bin/bash
# Round 5: k_encode straight 64-step blocks (no per-step tests where no step can need one,
# 32 x 64-bit remainder products, branch-free renormalisation) vs LAC_ENC_STRAIGHT=0
# (tools/_probe/liblac_base.so): the whole GPU suite, c2 and 64 / 256 streams, the c3 headline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05af}; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/gpu_tests.log 2>&1
rc=$?; tail -3 $o/gpu_tests.log; [ $rc -eq 0 ] || exit 3
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 5 --warmup 2 --decode-reps 3"
for r in 1 2 3; do
  timeout -k 10 200 $C2 > $o/c2_new$r.json 2> $o/c2_new$r.err || exit 3
  LAC_LIB=tools/_probe/liblac_base.so timeout -k 10 200 $C2 > $o/c2_base$r.json 2> $o/c2_base$r.err || exit 3
done
for s in 64 256; do
  timeout -k 10 200 python3 bench.py --cpu-baseline off --streams $s --tokens 1024 --steps 5 --warmup 2 --decode-reps 3 > $o/b${s}_new.json 2> $o/b${s}_new.err || exit 3
  LAC_LIB=tools/_probe/liblac_base.so timeout -k 10 200 python3 bench.py --cpu-baseline off --streams $s --tokens 1024 --steps 5 --warmup 2 --decode-reps 3 > $o/b${s}_base.json 2> $o/b${s}_base.err || exit 3
done
timeout -k 10 300 python3 bench.py > $o/c3_headline.json 2> $o/c3_headline.err || exit 3
for f in $o/c2_*.json $o/b*_*.json $o/c3_headline.json; do python3 -c "
import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']
print('$f'.split('/')[-1], 'enc %.3f M sym/s' % (d['value']/1e6), 'ms/step %.4f' % d['ms_per_step'], 'dec', p.get('decode',{}).get('symbols_per_s'), 'oracle', p.get('bit_exact_vs_oracle'))"; done
