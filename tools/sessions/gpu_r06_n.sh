#!/bin/bash
# Round 6: c2 with llama-scale u64 tables, the lean step's wide rows by division in the
# loads' shadow (LAC_LEAN_WIDE_DIV=1) against the product search (this tree), A/B x2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06n}; mkdir -p $o
LAC_LIB=tools/_probe/liblac_widediv.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_lean.py > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || exit 3
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 5 --warmup 2 --decode-reps 3 --pmf-bits 64"
for i in 1 2; do
  timeout -k 10 200 $C2 > $o/base_$i.json 2> $o/c2.err || exit 3
  LAC_LIB=tools/_probe/liblac_widediv.so timeout -k 10 200 $C2 > $o/wdiv_$i.json 2> $o/c2.err || exit 3
done
for f in base_1 wdiv_1 base_2 wdiv_2; do python3 -c "
import json; d=json.loads([l for l in open('$o/$f.json') if l.startswith('{')][-1]); p=d['parity']
print('$f', 'dec us/step %.3f' % (1e3*p['decode']['kernel_ms_per_step']), 'exact', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'))"; done
