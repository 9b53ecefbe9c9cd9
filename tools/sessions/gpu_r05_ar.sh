#!/bin/bash
# Round 5: the split encode path's row statistics overlapped with k_encode (a side stream
# computes the later pieces' statistics while the chain walks the first ones,
# LAC_ENC_OVERLAP) vs the previous commit: the whole GPU suite, c2 u32 x 3, c2 u64,
# 16 / 64 / 256 streams.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05ar}; mkdir -p $o
H=tools/_probe/liblac_head.so
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_straight.py tests/test_gpu_parity.py tests/test_gpu_checkpoint.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/gpu_tests.log 2>&1
rc=$?; tail -3 $o/gpu_tests.log; [ $rc -eq 0 ] || exit 3
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 5 --warmup 2 --decode-reps 2"
for r in 1 2 3; do
  timeout -k 10 200 $C2 > $o/c2_new$r.json 2> $o/c2_new$r.err || exit 3
  LAC_LIB=$H timeout -k 10 200 $C2 > $o/c2_head$r.json 2> $o/c2_head$r.err || exit 3
done
timeout -k 10 200 $C2 --pmf-bits 64 > $o/c2u64_new.json 2> $o/c2u64_new.err || exit 3
LAC_LIB=$H timeout -k 10 200 $C2 --pmf-bits 64 > $o/c2u64_head.json 2> $o/c2u64_head.err || exit 3
for s in 4 16 64; do
  B="python3 bench.py --cpu-baseline off --streams $s --tokens 1024 --steps 5 --warmup 2 --decode-reps 2"
  timeout -k 10 200 $B > $o/b${s}_new.json 2> $o/b${s}_new.err || exit 3
  LAC_LIB=$H timeout -k 10 200 $B > $o/b${s}_head.json 2> $o/b${s}_head.err || exit 3
done
for f in $o/c2*.json $o/b*_*.json; do python3 -c "
import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']
print('$f'.split('/')[-1], 'enc %.3f M sym/s' % (d['value']/1e6), 'ms/step %.4f' % d['ms_per_step'], 'exact', p['bit_exact_vs_oracle'], 'rt', p['round_trip_all_streams'])"; done
