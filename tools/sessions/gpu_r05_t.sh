#!/bin/bash
# Round 5: k_encode_pc (two waves per stream: chain + digit hand-off through LDS to a
# plane-appending wave; product for <= 1024 streams) vs k_encode (tools/_probe/liblac_nopc.so):
# the whole GPU suite, then c2 and 64 / 256 streams interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05t}; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/gpu_tests.log 2>&1
rc=$?; tail -3 $o/gpu_tests.log; [ $rc -eq 0 ] || exit 3
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 5 --warmup 2 --decode-reps 3"
for r in 1 2 3; do
  timeout -k 10 200 $C2 > $o/c2_pc$r.json 2> $o/c2_pc$r.err || exit 3
  LAC_LIB=tools/_probe/liblac_nopc.so timeout -k 10 200 $C2 > $o/c2_nopc$r.json 2> $o/c2_nopc$r.err || exit 3
done
for s in 64 256; do
  timeout -k 10 200 python3 bench.py --cpu-baseline off --streams $s --tokens 1024 --steps 5 --warmup 2 --decode-reps 3 > $o/b${s}_pc.json 2> $o/b${s}_pc.err || exit 3
  LAC_LIB=tools/_probe/liblac_nopc.so timeout -k 10 200 python3 bench.py --cpu-baseline off --streams $s --tokens 1024 --steps 5 --warmup 2 --decode-reps 3 > $o/b${s}_nopc.json 2> $o/b${s}_nopc.err || exit 3
done
for f in $o/c2_*.json $o/b*_*.json; do python3 -c "
import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']
print('$f'.split('/')[-1], 'enc %.3f M sym/s' % (d['value']/1e6), 'ms/step %.4f' % d['ms_per_step'], 'dec', p.get('decode',{}).get('symbols_per_s'), 'oracle', p.get('bit_exact_vs_oracle'))"; done
