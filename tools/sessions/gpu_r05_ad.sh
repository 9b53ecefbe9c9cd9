#!/bin/bash
# Round 5: k_decode_lean with its two-steps-ahead chunk-bounds prefetch issued after the
# step's own loads (LAC_LEAN_LATE_PF, product) vs before them (tools/_probe/liblac_earlypf.so);
# and k_q1_decode's next-step prefetch likewise (LAC_Q1DEC_LATE_PF, product) vs before its
# group loads (tools/_probe/liblac_q1early.so); the GPU suite first, then c2 and 4 / 16 / 64
# streams, then tools/q1_b2b.py at bf16 c3 / c4, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05ad}; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/gpu_tests.log 2>&1
rc=$?; tail -3 $o/gpu_tests.log; [ $rc -eq 0 ] || exit 3
for r in 1 2; do
  for v in new earlypf; do
    L=""; [ $v != new ] && L=tools/_probe/liblac_$v.so
    LAC_LIB=$L timeout -k 10 200 python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 3 --warmup 1 --decode-reps 5 > $o/c2_$v$r.json 2> $o/c2_$v$r.err || exit 3
  done
done
for s in 4 16 64; do
  for v in new earlypf; do
    L=""; [ $v != new ] && L=tools/_probe/liblac_$v.so
    LAC_LIB=$L timeout -k 10 200 python3 bench.py --cpu-baseline off --streams $s --tokens 512 --steps 3 --warmup 1 --decode-reps 5 > $o/b${s}_$v.json 2> $o/b${s}_$v.err || exit 3
  done
done
for V in 32000 128256; do
  for r in 1 2; do
    timeout -k 10 200 python3 tools/q1_b2b.py --vocab $V --reps 20 > $o/q1_new_${V}_$r.json 2> $o/q1_new_${V}_$r.err || exit 3
    LAC_LIB=tools/_probe/liblac_q1early.so timeout -k 10 200 python3 tools/q1_b2b.py --vocab $V --reps 20 > $o/q1_early_${V}_$r.json 2> $o/q1_early_${V}_$r.err || exit 3
  done
done
for f in $o/q1_*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); print('$f'.split('/')[-1], 'dec stats %.2f us/step' % (d['decode']['q1_stats_ms_per_launch']*1e3/16), 'q1dec %.2f' % d['decode']['q1_decode_us_per_step'])"; done
for f in $o/c2_*.json $o/b*_*.json; do python3 -c "
import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']; dd=p.get('decode',{})
print('$f'.split('/')[-1], 'dec %.1f k sym/s' % (dd.get('symbols_per_s')/1e3), {k: round(v*1e3,3) for k,v in (dd.get('kernel_ms_per_step_each') or {}).items()}, 'oracle', p.get('bit_exact_vs_oracle'))"; done
