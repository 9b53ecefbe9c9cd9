#!/bin/bash
# Round 6: L2-prefetching helper waves up to 44 streams (rows ahead fitted to 4 MB per XCD)
# against helpers up to 16 (tools/_probe/liblac_help16.so): 1 / 16 / 24 / 32 / 44 streams,
# V=32000 u32, 1024 steps, and the c2 u64 line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06ac}; mkdir -p $o
for b in 1 16 24 32 44; do
for v in default help16; do
    if [ $v = default ]; then L=""; else L=tools/_probe/liblac_$v.so; fi
    LAC_LIB=$L timeout -k 10 200 python3 bench.py --cpu-baseline off --streams $b --tokens 1024 --steps 3 --warmup 1 --decode-reps 3 > $o/${v}_b$b.json 2> $o/${v}_b$b.err || exit 3
done
done
for v in default help16; do
    if [ $v = default ]; then L=""; else L=tools/_probe/liblac_$v.so; fi
    LAC_LIB=$L timeout -k 10 200 python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 3 --warmup 1 --decode-reps 3 --pmf-bits 64 > $o/${v}_c2u64.json 2> $o/${v}_c2u64.err || exit 3
done
for f in $o/*.json; do python3 -c "
import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']
print('$(basename $f)', 'dec %.2f M sym/s' % (p['decode']['symbols_per_s']/1e6), 'dec us/step %.3f' % (1e3*p['decode']['kernel_ms_per_step']), 'exact', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'))"; done
