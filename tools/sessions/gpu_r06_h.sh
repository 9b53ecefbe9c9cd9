#!/bin/bash
# Round 6: lean step with the LeanMeta by vector load (lean tests, c2 u32/u64, drop-in,
# phases incl. a static u64 row of ~2^40 totals), then the bf16 c3 logits row-stats
# variants A/B: late tail, roll-first, both (tools/q1_b2b.py, liblac hipEvents).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06h}; mkdir -p $o
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_lean.py tests/test_gpu_dropin.py > $o/lean.log 2>&1
rc=$?; tail -2 $o/lean.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python3 tools/dropin_bench.py --out $o/dropin.json > $o/dropin.log 2>&1 || exit 3
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 5 --warmup 2 --decode-reps 3"
timeout -k 10 200 $C2 > $o/c2_1.json 2> $o/c2.err || exit 3
timeout -k 10 200 $C2 --pmf-bits 64 > $o/c2_u64.json 2> $o/c2_u64.err || exit 3
timeout -k 10 200 $C2 > $o/c2_2.json 2> $o/c2.err || exit 3
P="python3 tools/dec_phase_probe.py"
LAC_LIB=tools/_probe/liblac_phases.so timeout -k 10 120 $P > $o/phases_c2.json 2>> $o/err.log || exit 3
LAC_LIB=tools/_probe/liblac_phases.so timeout -k 10 120 $P --pmf-bits 64 > $o/phases_c2_u64.json 2>> $o/err.log || exit 3
LAC_LIB=tools/_probe/liblac_phases.so timeout -k 10 120 $P --pmf-bits 64 --scale-bits 40 --static > $o/phases_static40_u64.json 2>> $o/err.log || exit 3
cat $o/dropin.json $o/phases_*.json
for f in c2_1 c2_2 c2_u64; do python3 -c "
import json; d=json.loads([l for l in open('$o/$f.json') if l.startswith('{')][-1]); p=d['parity']
print('$f', '%.3f M sym/s' % (d['value']/1e6), 'dec %.3f M' % (p['decode']['symbols_per_s']/1e6), 'dec us/step %.3f' % (1e3*p['decode']['kernel_ms_per_step']), 'exact', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'))"; done
for v in late rollfirst late_rf; do
  LAC_LIB=tools/_probe/liblac_$v.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
      tests/test_gpu_logits.py -k "c3 or shape or bf16" > $o/t_$v.log 2>&1
  rc=$?; tail -1 $o/t_$v.log; [ $rc -eq 0 ] || exit 3
done
for i in 1 2; do
  timeout -k 10 120 python3 tools/q1_b2b.py --vocab 32000 --reps 20 > $o/q_base_$i.json 2>> $o/err.log || exit 3
  for v in late rollfirst late_rf; do
    LAC_LIB=tools/_probe/liblac_$v.so timeout -k 10 120 python3 tools/q1_b2b.py --vocab 32000 --reps 20 > $o/q_${v}_$i.json 2>> $o/err.log || exit 3
  done
done
for f in $o/q_*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); print('$f', {k: (round(v['q1_stats_ms_per_launch']*1e3/16, 2), round(v['frac_of_8TBps'], 4), v.get('q1_decode_us_per_step') and round(v['q1_decode_us_per_step'], 2)) for k, v in d.items() if isinstance(v, dict)})"; done
