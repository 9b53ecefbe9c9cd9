#!/bin/bash
# Round 6: the lean buffers' size (LAC_LEAN_BYTES: 256 MB kept, 512 MB, 1 GB): more rows per
# launch group make the stats pass run more waves per CU.  c2 u32 / u64 decode lines, twice,
# plus a kernel trace of each c2 decode at 1 GB.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06w}; mkdir -p $o
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 3 --warmup 1 --decode-reps 3"
for rep in 1 2; do
for v in default lb512 lb1g; do
    if [ $v = default ]; then L=""; else L=tools/_probe/liblac_$v.so; fi
    LAC_LIB=$L timeout -k 10 200 $C2 > $o/${v}_u32_$rep.json 2> $o/${v}.err || exit 3
    LAC_LIB=$L timeout -k 10 200 $C2 --pmf-bits 64 > $o/${v}_u64_$rep.json 2> $o/${v}.err || exit 3
done
done
for f in $o/*.json; do python3 -c "
import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']
print('$(basename $f)', 'dec us/step %.3f' % (1e3*p['decode']['kernel_ms_per_step']), 'exact', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'))"; done
