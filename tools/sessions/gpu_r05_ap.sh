#!/bin/bash
# Round 5: the lean decoder's L2-prefetch helpers re-tuned for the faster step (1.116 us):
# rows ahead 16 (product) / 24 / 32, and 32 helper waves per stream; c2 decode, 3 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05ap}; mkdir -p $o
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 2 --warmup 1 --decode-reps 5"
for r in 1 2 3; do
  for lib in prod ahead24 ahead32 help32; do
    if [ $lib = prod ]; then L=""; else L=tools/_probe/liblac_$lib.so; fi
    LAC_LIB=$L timeout -k 10 200 $C2 > $o/c2_${lib}_$r.json 2> $o/c2_${lib}_$r.err || exit 3
  done
done
for f in $o/c2_*.json; do python3 -c "
import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']; dd=p['decode']
print('$f'.split('/')[-1], 'dec us/step %.4f' % (dd['kernel_ms_per_step']*1e3), 'rt', p['round_trip_all_streams'], 'exact', p['bit_exact_vs_oracle'])"; done
