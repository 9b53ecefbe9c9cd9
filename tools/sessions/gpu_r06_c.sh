#!/bin/bash
# Round 6: per-entry-CDF lean decode (u32 + u64 tables), static rows' statistics once per
# stream, LAC_OPT_DECODE_STOP in the drop-in static decode: the whole GPU suite, then the
# drop-in line, c2 u32 / u64 lines and the --gather line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06c}; mkdir -p $o
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_lean.py > $o/lean.log 2>&1
rc=$?; tail -3 $o/lean.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/gpu_tests.log 2>&1
rc=$?; tail -3 $o/gpu_tests.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python3 tools/dropin_bench.py --out $o/dropin.json > $o/dropin.log 2>&1 || exit 3
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 5 --warmup 2 --decode-reps 3"
timeout -k 10 200 $C2 > $o/c2.json 2> $o/c2.err || exit 3
timeout -k 10 200 $C2 --pmf-bits 64 > $o/c2_u64.json 2> $o/c2_u64.err || exit 3
timeout -k 10 300 python3 bench.py --gather --cpu-baseline off > $o/gather_w1.json 2> $o/gather_w1.err || exit 3
cat $o/dropin.json
for f in c2 c2_u64 gather_w1; do python3 -c "
import json; d=json.loads([l for l in open('$o/$f.json') if l.startswith('{')][-1]); p=d['parity']
print('$f', '%.3f M sym/s' % (d['value']/1e6), 'dec %.3f M' % (p['decode']['symbols_per_s']/1e6), 'dec us/step %.3f' % (1e3*p['decode']['kernel_ms_per_step']), 'exact', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'), 'gather', p.get('gather_ok'), p.get('gather'))"; done
