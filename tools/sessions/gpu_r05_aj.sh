#!/bin/bash
# Round 5: the generalised straight blocks with 32-bit row fields and a flag for the fudge
# exit vs the previous commit: encode parity tests, c2 u32 x 3 and u64 x 2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05aj}; mkdir -p $o
H=tools/_probe/liblac_head.so
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_checkpoint.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/gpu_tests.log 2>&1
rc=$?; tail -3 $o/gpu_tests.log; [ $rc -eq 0 ] || exit 3
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 5 --warmup 2 --decode-reps 3"
for r in 1 2 3; do
  timeout -k 10 200 $C2 > $o/c2_new$r.json 2> $o/c2_new$r.err || exit 3
  LAC_LIB=$H timeout -k 10 200 $C2 > $o/c2_head$r.json 2> $o/c2_head$r.err || exit 3
done
for r in 1 2; do
  timeout -k 10 200 $C2 --pmf-bits 64 > $o/c2u64_new$r.json 2> $o/c2u64_new$r.err || exit 3
  LAC_LIB=$H timeout -k 10 200 $C2 --pmf-bits 64 > $o/c2u64_head$r.json 2> $o/c2u64_head$r.err || exit 3
done
for f in $o/c2*.json; do python3 -c "
import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']; dd=p.get('decode',{})
print('$f'.split('/')[-1], 'enc %.3f M sym/s' % (d['value']/1e6), 'ms/step %.4f' % d['ms_per_step'], 'dec %.3f M' % (dd.get('symbols_per_s',0)/1e6), 'oracle', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'))"; done
