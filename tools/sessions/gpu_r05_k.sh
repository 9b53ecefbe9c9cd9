#!/bin/bash
# Round 5: permlane cross-row sums (logits tests + b2b A/B vs the round-start form),
# and why the bench's k_q1_decode per-step time differs from q1_b2b's (reps 5 vs 20).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05k}; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_logits.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/t.log 2>&1
rc=$?; tail -3 $o/t.log; [ $rc -eq 0 ] || exit 3
for r in 1 2; do
  timeout -k 10 200 python3 tools/q1_b2b.py --vocab 32000 --reps 20 > $o/b2b_new$r.json 2> $o/b2b_new$r.err || exit 3
  LAC_LIB=tools/_probe/liblac_nodefer.so timeout -k 10 200 python3 tools/q1_b2b.py --vocab 32000 --reps 20 > $o/b2b_base$r.json 2> $o/b2b_base$r.err || exit 3
done
timeout -k 10 200 python3 tools/q1_b2b.py --vocab 32000 --reps 5 > $o/b2b_reps5.json 2> $o/b2b_reps5.err || exit 3
for f in $o/b2b_*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); print('$f'.split('/')[-1], 'enc %.1f us/step' % (d['encode']['q1_stats_ms_per_launch']*1e3/16), 'dec %.1f us/step' % (d['decode']['q1_stats_ms_per_launch']*1e3/16), 'dec2 %.1f' % (d['decode2']['q1_stats_ms_per_launch']*1e3/16), 'q1dec %.2f %.2f' % (d['decode']['q1_decode_us_per_step'], d['decode2']['q1_decode_us_per_step']))"; done
timeout -k 10 200 python3 bench.py --input logits-bf16 --steps 20 --warmup 3 --cpu-baseline off --decode-reps 5 > $o/bf16c3_r5.json 2> $o/bf16c3_r5.err || exit 3
timeout -k 10 200 python3 bench.py --input logits-bf16 --steps 20 --warmup 3 --cpu-baseline off --decode-reps 20 > $o/bf16c3_r20.json 2> $o/bf16c3_r20.err || exit 3
for f in bf16c3_r5 bf16c3_r20; do python3 -c "
import json
j=json.loads([l for l in open('$o/$f.json') if l.startswith('{')][-1])
r=j['roofline'];d=j['parity']['decode']
print('$f', round(j['value']/1e6,2), round(r['kernel_ms_per_launch'],4), round(r['frac'],3), 'dec', round(d['symbols_per_s']/1e6,2), {k:round(v*1e3,2) for k,v in d['kernel_ms_per_step_each'].items()})
"; done
