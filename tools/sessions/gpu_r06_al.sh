#!/bin/bash
# Round 6: one-stream decode across vocabularies, u32 and llama-scale u64 tables, 2048 steps:
# V = 1000 / 32000 / 65536 (u64 rows of 65536 entries take the lean step since the two
# chunk bounds per lane; before, k_decode_seq).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06al}; mkdir -p $o
for v in 1000 32000 65536; do
for bits in 32 64; do
    timeout -k 10 200 python3 bench.py --cpu-baseline off --streams 1 --tokens 2048 --vocab $v --pmf-bits $bits --steps 3 --warmup 1 --decode-reps 3 > $o/v${v}_u$bits.json 2> $o/v${v}_u$bits.err || exit 3
done
done
for f in $o/*.json; do python3 -c "
import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']
print('$(basename $f)', 'enc %.2f M sym/s' % (d['value']/1e6), 'dec %.3f M sym/s' % (p['decode']['symbols_per_s']/1e6), 'dec us/step %.3f' % (1e3*p['decode']['kernel_ms_per_step']), 'exact', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'))"; done
