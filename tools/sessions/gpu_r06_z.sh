#!/bin/bash
# Round 6: the few-stream decode after the lean step's second pass, V=32000 u32, 1024 steps:
# 1 / 4 / 16 / 64 / 128 / 256 streams (lean step up to 64, helpers up to 16; then k_decode_seq
# and the block path), and 64 / 128 / 256 streams with the lean step allowed up to 256
# (tools/_probe/liblac_lean256.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06z}; mkdir -p $o
for b in 1 4 16 64 128 256; do
    timeout -k 10 200 python3 bench.py --cpu-baseline off --streams $b --tokens 1024 --steps 3 --warmup 1 --decode-reps 3 > $o/b$b.json 2> $o/b$b.err || exit 3
done
for b in 64 128 256; do
    LAC_LIB=tools/_probe/liblac_lean256.so timeout -k 10 200 python3 bench.py --cpu-baseline off --streams $b --tokens 1024 --steps 3 --warmup 1 --decode-reps 3 > $o/lean256_b$b.json 2> $o/lean256_b$b.err || exit 3
done
for b in 1 4 16 64 128 256; do python3 -c "
import json; d=json.loads([l for l in open('$o/b$b.json') if l.startswith('{')][-1]); p=d['parity']
print('B=$b', 'enc %.2f M sym/s' % (d['value']/1e6), 'dec %.2f M sym/s' % (p['decode']['symbols_per_s']/1e6), 'dec us/step %.3f' % (1e3*p['decode']['kernel_ms_per_step']), 'exact', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'))"; done
for b in 64 128 256; do python3 -c "
import json; d=json.loads([l for l in open('$o/lean256_b$b.json') if l.startswith('{')][-1]); p=d['parity']
print('lean256 B=$b', 'dec %.2f M sym/s' % (p['decode']['symbols_per_s']/1e6), 'dec us/step %.3f' % (1e3*p['decode']['kernel_ms_per_step']), 'exact', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'))"; done
