#!/bin/bash
# Round 6: the helpers' rows ahead fitted to 2 MB per XCD when several streams share one
# (tools/_probe/liblac_ah2m.so: 8 rows at 2 streams per XCD, 4 at 4) against 16 for all:
# 12 / 16 streams (V=32000 u32, 1024 steps), twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06ak}; mkdir -p $o
for rep in 1 2; do
for b in 12 16; do
for v in default ah2m; do
    if [ $v = default ]; then L=""; else L=tools/_probe/liblac_$v.so; fi
    LAC_LIB=$L timeout -k 10 200 python3 bench.py --cpu-baseline off --streams $b --tokens 1024 --steps 3 --warmup 1 --decode-reps 3 > $o/${v}_b${b}_$rep.json 2> $o/${v}.err || exit 3
done
done
done
for f in $o/*.json; do python3 -c "
import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']
print('$(basename $f)', 'dec %.2f M sym/s' % (p['decode']['symbols_per_s']/1e6), 'dec us/step %.3f' % (1e3*p['decode']['kernel_ms_per_step']), 'exact', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'))"; done
