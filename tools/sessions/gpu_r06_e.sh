#!/bin/bash
# Round 6: bf16 c3 logits row statistics: the CONTIG vector layout
# (wave w holds 8 consecutive 64-vector groups, one contiguous chunk-total store) against
# the strided one, back to back on one box (tools/q1_b2b.py, liblac hipEvents), after the
# logits parity tests on the variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06e}; mkdir -p $o
P="python3 tools/dec_phase_probe.py"
LAC_LIB=tools/_probe/liblac_phases.so timeout -k 10 120 $P > $o/phases_c2.json 2>> $o/err.log || exit 3
LAC_LIB=tools/_probe/liblac_phases.so timeout -k 10 120 $P --pmf-bits 64 > $o/phases_c2_u64.json 2>> $o/err.log || exit 3
LAC_LIB=tools/_probe/liblac_phases.so timeout -k 10 120 $P --pmf-bits 64 --static > $o/phases_static_u64.json 2>> $o/err.log || exit 3
LAC_LIB=tools/_probe/liblac_phases.so timeout -k 10 120 $P --static > $o/phases_static_u32.json 2>> $o/err.log || exit 3
timeout -k 10 120 $P --pmf-bits 64 --static > $o/plain_static_u64.json 2>> $o/err.log || exit 3
cat $o/phases_*.json $o/plain_static_u64.json
LAC_LIB=tools/_probe/liblac_contig.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_logits.py > $o/contig_tests.log 2>&1
rc=$?; tail -2 $o/contig_tests.log; [ $rc -eq 0 ] || exit 3
for i in 1 2 3; do
  timeout -k 10 120 python3 tools/q1_b2b.py --vocab 32000 --reps 20 > $o/base_$i.json 2>> $o/err.log || exit 3
  LAC_LIB=tools/_probe/liblac_contig.so timeout -k 10 120 python3 tools/q1_b2b.py --vocab 32000 --reps 20 > $o/contig_$i.json 2>> $o/err.log || exit 3
done
for f in $o/base_*.json $o/contig_*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); print('$f', {k: (round(v['q1_stats_ms_per_launch']*1e3/16, 2), round(v['frac_of_8TBps'], 4), v.get('q1_decode_us_per_step') and round(v['q1_decode_us_per_step'], 2)) for k, v in d.items() if isinstance(v, dict)})"; done
