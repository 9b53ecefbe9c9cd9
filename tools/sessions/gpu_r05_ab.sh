#!/bin/bash
# Round 5: the c2 lean decode -- the decoder's progress store (for its L2-prefetching
# helpers) every 8 steps (product) vs 16 / 32 (tools/_probe/liblac_pub16.so, _pub32.so)
# and no helpers at all (_nohelp.so); c2 bench lines interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05ab}; mkdir -p $o
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 3 --warmup 1 --decode-reps 5"
for r in 1 2; do
  for v in new pub16 pub32 nohelp; do
    L=""; [ $v != new ] && L=tools/_probe/liblac_$v.so
    LAC_LIB=$L timeout -k 10 200 $C2 > $o/c2_$v$r.json 2> $o/c2_$v$r.err || exit 3
  done
done
for f in $o/c2_*.json; do python3 -c "
import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']; dd=p.get('decode',{})
print('$f'.split('/')[-1], 'dec %.1f k sym/s' % (dd.get('symbols_per_s')/1e3), {k: round(v*1e3,3) for k,v in (dd.get('kernel_ms_per_step_each') or {}).items()}, 'oracle', p.get('bit_exact_vs_oracle'))"; done
