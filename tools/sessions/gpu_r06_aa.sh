#!/bin/bash
# Round 6: where the lean step stops paying with the per-entry CDF (its stats pass writes a
# full CDF copy): 8 / 16 / 32 / 64 streams, V=32000 u32, 1024 steps, the kept build (lean up
# to 64 streams) against one with the lean step only up to 4 (tools/_probe/liblac_lean4.so:
# k_dec_stats + k_decode_seq above).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06aa}; mkdir -p $o
for b in 8 16 32 64; do
for v in default lean4; do
    if [ $v = default ]; then L=""; else L=tools/_probe/liblac_$v.so; fi
    LAC_LIB=$L timeout -k 10 200 python3 bench.py --cpu-baseline off --streams $b --tokens 1024 --steps 3 --warmup 1 --decode-reps 3 > $o/${v}_b$b.json 2> $o/${v}_b$b.err || exit 3
done
done
for f in $o/*.json; do python3 -c "
import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']
print('$(basename $f)', 'dec %.2f M sym/s' % (p['decode']['symbols_per_s']/1e6), 'dec us/step %.3f' % (1e3*p['decode']['kernel_ms_per_step']), 'exact', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'))"; done
