#!/bin/bash
# Round 5: k_q1_decode with fast rows re-quantised without the cap (packed FMAs,
# LAC_Q1D_FAST) and the renormalisation without branches (decode_advance_nb, LAC_Q1D_NB),
# each alone and both, vs the previous commit: logits GPU tests, then tools/q1_b2b.py
# (bf16, 4096 streams, 20 passes back to back) at V = 32000 and 128256, interleaved; and
# k_decode_seq with the same renormalisation (c2 with u64 tables, decode).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05al}; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_logits.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_flush.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/gpu_tests.log 2>&1
rc=$?; tail -3 $o/gpu_tests.log; [ $rc -eq 0 ] || exit 3
for r in 1 2; do
  for V in 32000 128256; do
    for lib in head q1nofast q1nonb new; do
      if [ $lib = new ]; then L=""; else L=tools/_probe/liblac_$lib.so; fi
      LAC_LIB=$L timeout -k 10 200 python3 tools/q1_b2b.py --vocab $V --reps 20 > $o/b2b_${lib}_${V}_$r.json 2> $o/b2b_${lib}_${V}_$r.err || exit 3
    done
  done
done
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 3 --warmup 1 --decode-reps 3 --pmf-bits 64"
for r in 1 2; do
  timeout -k 10 200 $C2 > $o/c2u64_new$r.json 2> $o/c2u64_new$r.err || exit 3
  LAC_LIB=tools/_probe/liblac_head.so timeout -k 10 200 $C2 > $o/c2u64_head$r.json 2> $o/c2u64_head$r.err || exit 3
done
for f in $o/c2u64_*.json; do python3 -c "
import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']; dd=p['decode']
print('$f'.split('/')[-1], 'dec %.4f M sym/s' % (dd['symbols_per_s']/1e6), {k: round(v*1e3,3) for k,v in dd['kernel_ms_per_step_each'].items()}, 'exact', p['bit_exact_vs_oracle'], 'rt', p['round_trip_all_streams'])"; done
for f in $o/b2b_*.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f'.split('/')[-1], 'dec stats %.2f us' % (d['decode2']['q1_stats_ms_per_launch']*1e3/16), 'q1_decode %.3f us/step' % d['decode2']['q1_decode_us_per_step'], d['decode2'].get('round_trip'))"; done
