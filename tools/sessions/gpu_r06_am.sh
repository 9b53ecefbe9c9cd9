#!/bin/bash
# Round 6: the helpers' rows ahead capped at 4 MB per XCD (u64 rows of 65536 entries: 8 rows
# instead of 16) against no cap (tools/_probe/liblac_ahinf.so): one stream, 2048 steps,
# V = 65536 u64 and u32 and V = 32000 u64, twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06am}; mkdir -p $o
for rep in 1 2; do
for cfg in "65536 64" "65536 32" "32000 64"; do
set -- $cfg
for v in default ahinf; do
    if [ $v = default ]; then L=""; else L=tools/_probe/liblac_$v.so; fi
    LAC_LIB=$L timeout -k 10 200 python3 bench.py --cpu-baseline off --streams 1 --tokens 2048 --vocab $1 --pmf-bits $2 --steps 3 --warmup 1 --decode-reps 3 > $o/${v}_v$1_u$2_$rep.json 2> $o/${v}.err || exit 3
done
done
done
for f in $o/*.json; do python3 -c "
import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']
print('$(basename $f)', 'dec us/step %.3f' % (1e3*p['decode']['kernel_ms_per_step']), 'exact', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'))"; done
