#!/bin/bash
# Round 5: some processes run the bf16 c3 decode form of the row statistics at 39.1-39.5
# us per step, most at 42.1-42.4 (gpu_r05_al.sh), with the same code: is it where the
# chunk-total buffer lands?  The product vs the buffer offset by 64 KB + 256 B and by
# 1 MB + 4 KB (LAC_Q1CH_PAD probe builds), tools/q1_b2b.py at V = 32000, 4 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05am}; mkdir -p $o
for r in 1 2 3 4; do
  for lib in prod pad64k pad1m; do
    if [ $lib = prod ]; then L=""; else L=tools/_probe/liblac_$lib.so; fi
    LAC_LIB=$L timeout -k 10 200 python3 tools/q1_b2b.py --vocab 32000 --reps 20 > $o/b2b_${lib}_$r.json 2> $o/b2b_${lib}_$r.err || exit 3
  done
done
for f in $o/b2b_*.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f'.split('/')[-1], ' '.join('%s %.2f' % (k, d[k]['q1_stats_ms_per_launch']*1e3/16) for k in ('encode','decode','encode2','decode2')), 'q1dec %.3f' % d['decode2']['q1_decode_us_per_step'], d['decode2'].get('round_trip'))"; done
