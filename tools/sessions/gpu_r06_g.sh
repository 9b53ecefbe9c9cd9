#!/bin/bash
# Round 6: the lean step unrolled 2x (prefetch registers touched two steps after their
# loads), static rows without per-step reloads, u64 search by products; lean + drop-in
# tests, the drop-in line, c2 u32 / u64 lines (and u32 with the product search, A/B).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06g}; mkdir -p $o
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_lean.py tests/test_gpu_dropin.py tests/test_gpu_flush.py > $o/lean.log 2>&1
rc=$?; tail -2 $o/lean.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python3 tools/dropin_bench.py --out $o/dropin.json > $o/dropin.log 2>&1 || exit 3
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 5 --warmup 2 --decode-reps 3"
for i in 1 2; do
timeout -k 10 200 $C2 > $o/c2_$i.json 2> $o/c2.err || exit 3
LAC_LIB=tools/_probe/liblac_prod32.so timeout -k 10 200 $C2 > $o/c2p_$i.json 2> $o/c2p.err || exit 3
done
timeout -k 10 200 $C2 --pmf-bits 64 > $o/c2_u64.json 2> $o/c2_u64.err || exit 3
P="python3 tools/dec_phase_probe.py"
LAC_LIB=tools/_probe/liblac_phases.so timeout -k 10 120 $P > $o/phases_c2.json 2>> $o/err.log || exit 3
LAC_LIB=tools/_probe/liblac_phases.so timeout -k 10 120 $P --pmf-bits 64 > $o/phases_c2_u64.json 2>> $o/err.log || exit 3
cat $o/dropin.json $o/phases_*.json
for f in c2_1 c2p_1 c2_2 c2p_2 c2_u64; do python3 -c "
import json; d=json.loads([l for l in open('$o/$f.json') if l.startswith('{')][-1]); p=d['parity']
print('$f', '%.3f M sym/s' % (d['value']/1e6), 'dec %.3f M' % (p['decode']['symbols_per_s']/1e6), 'dec us/step %.3f' % (1e3*p['decode']['kernel_ms_per_step']), 'exact', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'))"; done
