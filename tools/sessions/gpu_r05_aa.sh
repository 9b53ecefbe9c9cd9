#!/bin/bash
# Round 5: k_q1_decode with the symbol inside the crossing lane picked on the scalar unit
# (LAC_Q1DEC_SCALAR_PICK, product) vs every lane's vector pick (tools/_probe/liblac_vpick.so);
# logits / fuzz suites first, tools/q1_b2b.py at bf16 c3 / c4 / Qwen2 interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05aa}; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_logits.py tests/test_gpu_fuzz.py tests/test_gpu_api.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/t.log 2>&1
rc=$?; tail -3 $o/t.log; [ $rc -eq 0 ] || exit 3
for V in 32000 128256 151936; do
  for r in 1 2; do
    timeout -k 10 200 python3 tools/q1_b2b.py --vocab $V --reps 20 > $o/b2b_new_${V}_$r.json 2> $o/b2b_new_${V}_$r.err || exit 3
    LAC_LIB=tools/_probe/liblac_vpick.so timeout -k 10 200 python3 tools/q1_b2b.py --vocab $V --reps 20 > $o/b2b_base_${V}_$r.json 2> $o/b2b_base_${V}_$r.err || exit 3
  done
done
for f in $o/b2b_*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); print('$f'.split('/')[-1], 'dec stats %.2f us/step' % (d['decode']['q1_stats_ms_per_launch']*1e3/16), 'q1dec %.2f' % d['decode']['q1_decode_us_per_step'])"; done
