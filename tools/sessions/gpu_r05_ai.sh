#!/bin/bash
# Round 5: k_encode's straight blocks for 64-bit totals (T < 2^62) and rows that can fudge
# (a fudged step leaves for the general step) vs the previous commit
# (tools/_probe/liblac_head.so): the whole GPU suite, c2 with u32 and with u64 llama-scale
# tables, 64 streams u64, the drop-in surface (tools/dropin_bench.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05ai}; mkdir -p $o
H=tools/_probe/liblac_head.so
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/gpu_tests.log 2>&1
rc=$?; tail -3 $o/gpu_tests.log; [ $rc -eq 0 ] || exit 3
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 5 --warmup 2 --decode-reps 3"
for r in 1 2; do
  timeout -k 10 200 $C2 > $o/c2_new$r.json 2> $o/c2_new$r.err || exit 3
  LAC_LIB=$H timeout -k 10 200 $C2 > $o/c2_head$r.json 2> $o/c2_head$r.err || exit 3
  timeout -k 10 200 $C2 --pmf-bits 64 > $o/c2u64_new$r.json 2> $o/c2u64_new$r.err || exit 3
  LAC_LIB=$H timeout -k 10 200 $C2 --pmf-bits 64 > $o/c2u64_head$r.json 2> $o/c2u64_head$r.err || exit 3
done
B="python3 bench.py --cpu-baseline off --streams 64 --tokens 1024 --steps 5 --warmup 2 --decode-reps 3 --pmf-bits 64"
timeout -k 10 200 $B > $o/b64u64_new.json 2> $o/b64u64_new.err || exit 3
LAC_LIB=$H timeout -k 10 200 $B > $o/b64u64_head.json 2> $o/b64u64_head.err || exit 3
timeout -k 10 300 python3 tools/dropin_bench.py --out $o/dropin_new.json > $o/dropin_new.log 2>&1 || exit 3
LAC_LIB=$H timeout -k 10 300 python3 tools/dropin_bench.py --out $o/dropin_head.json > $o/dropin_head.log 2>&1 || exit 3
for f in $o/c2*.json $o/b64*.json; do python3 -c "
import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']; dd=p.get('decode',{})
print('$f'.split('/')[-1], 'enc %.3f M sym/s' % (d['value']/1e6), 'ms/step %.4f' % d['ms_per_step'], 'dec %.3f M' % (dd.get('symbols_per_s',0)/1e6), 'oracle', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'), 'fudge', p.get('rows_that_can_fudge'))"; done
tail -c 600 $o/dropin_new.json; echo; tail -c 600 $o/dropin_head.json
