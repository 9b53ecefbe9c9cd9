#!/bin/bash
# Round 5: k_encode's step inputs by scalar loads (LAC_ENC_PRE, product: k_row_stats stores
# the row fractions, each step's 64-B RowStats + symbol arrive in SGPRs one step ahead) vs
# the lane prefetch + readlanes (tools/_probe/liblac_nopre.so): the whole GPU suite, c2
# (one stream x 4096 steps) and 64 / 256 streams interleaved, and the phase probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05s}; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/gpu_tests.log 2>&1
rc=$?; tail -3 $o/gpu_tests.log; [ $rc -eq 0 ] || exit 3
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 5 --warmup 2 --decode-reps 3"
for r in 1 2 3; do
  timeout -k 10 200 $C2 > $o/c2_pre$r.json 2> $o/c2_pre$r.err || exit 3
  LAC_LIB=tools/_probe/liblac_nopre.so timeout -k 10 200 $C2 > $o/c2_nopre$r.json 2> $o/c2_nopre$r.err || exit 3
done
for s in 64 256; do
  timeout -k 10 200 python3 bench.py --cpu-baseline off --streams $s --tokens 1024 --steps 5 --warmup 2 --decode-reps 3 > $o/b${s}_pre.json 2> $o/b${s}_pre.err || exit 3
  LAC_LIB=tools/_probe/liblac_nopre.so timeout -k 10 200 python3 bench.py --cpu-baseline off --streams $s --tokens 1024 --steps 5 --warmup 2 --decode-reps 3 > $o/b${s}_nopre.json 2> $o/b${s}_nopre.err || exit 3
done
LAC_LIB=tools/_probe/liblac_encphases.so timeout -k 10 200 python3 tools/enc_phase_probe.py > $o/enc_phases.json 2> $o/enc_phases.err || exit 3
cat $o/enc_phases.json | cut -c1-600
for f in $o/c2_*.json $o/b*_*.json; do python3 -c "
import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']
print('$f'.split('/')[-1], 'enc %.3f M sym/s' % (d['value']/1e6), 'ms/step %.4f' % d['ms_per_step'], 'dec', p.get('decode',{}).get('symbols_per_s'), 'oracle', p.get('bit_exact_vs_oracle'))"; done
