#!/bin/bash
# Round 5: k_q1_decode with loop-local registers, prefix chunk sums from k_q1_stats and
# the fast re-quantisation: logits/fuzz/api GPU tests, then q1_b2b new vs the round's
# earlier library (tools/_probe/liblac_presplit.so) at bf16 c3 / c4 / Qwen2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05n}; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_logits.py tests/test_gpu_fuzz.py tests/test_gpu_api.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/t.log 2>&1
rc=$?; tail -3 $o/t.log; [ $rc -eq 0 ] || exit 3
for V in 32000 128256 151936; do
  for r in 1 2; do
    timeout -k 10 200 python3 tools/q1_b2b.py --vocab $V --reps 20 > $o/b2b_new_${V}_$r.json 2> $o/b2b_new_${V}_$r.err || exit 3
    LAC_LIB=tools/_probe/liblac_presplit.so timeout -k 10 200 python3 tools/q1_b2b.py --vocab $V --reps 20 > $o/b2b_base_${V}_$r.json 2> $o/b2b_base_${V}_$r.err || exit 3
  done
done
for f in $o/b2b_*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); print('$f'.split('/')[-1], 'dec stats %.1f us/step' % (d['decode']['q1_stats_ms_per_launch']*1e3/16), 'q1dec %.2f %.2f' % (d['decode']['q1_decode_us_per_step'], d['decode2']['q1_decode_us_per_step']), d['decode']['round_trip'])"; done
timeout -k 10 200 python3 bench.py --input logits-bf16 --steps 20 --warmup 3 --cpu-baseline off > $o/bf16c3.json 2> $o/bf16c3.err || exit 3
python3 -c "
import json
j=json.loads([l for l in open('$o/bf16c3.json') if l.startswith('{')][-1])
d=j['parity']['decode']; print('bench bf16 c3', round(j['value']/1e6,2), 'dec', round(d['symbols_per_s']/1e6,2), d['kernel_ms_per_step_each'], j['parity']['round_trip_all_streams'], j['parity']['bit_exact_vs_oracle'])"
