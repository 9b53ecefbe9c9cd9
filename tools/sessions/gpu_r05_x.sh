#!/bin/bash
# Round 5: k_encode -- quotients for 32-bit totals by one double estimate + a sign-mask
# correction (LAC_ENC_DIV32) and the prefetch waited for before the step loop
# (LAC_ENC_PREWAIT): product vs div32 only (tools/_probe/liblac_div32.so) vs the previous
# commit (tools/_probe/liblac_base.so); the whole GPU suite first, the c3 headline last.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05x}; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/gpu_tests.log 2>&1
rc=$?; tail -3 $o/gpu_tests.log; [ $rc -eq 0 ] || exit 3
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 5 --warmup 2 --decode-reps 3"
for r in 1 2 3; do
  timeout -k 10 200 $C2 > $o/c2_new$r.json 2> $o/c2_new$r.err || exit 3
  LAC_LIB=tools/_probe/liblac_div32.so timeout -k 10 200 $C2 > $o/c2_div32$r.json 2> $o/c2_div32$r.err || exit 3
  LAC_LIB=tools/_probe/liblac_base.so timeout -k 10 200 $C2 > $o/c2_base$r.json 2> $o/c2_base$r.err || exit 3
done
for s in 64 256; do
  for v in new base; do
    L=""; [ $v = base ] && L=tools/_probe/liblac_base.so
    LAC_LIB=$L timeout -k 10 200 python3 bench.py --cpu-baseline off --streams $s --tokens 1024 --steps 5 --warmup 2 --decode-reps 3 > $o/b${s}_$v.json 2> $o/b${s}_$v.err || exit 3
  done
done
timeout -k 10 300 python3 bench.py > $o/c3_headline.json 2> $o/c3_headline.err || exit 3
timeout -k 10 300 python3 bench.py --input logits-bf16 --cpu-baseline off > $o/bf16_c3.json 2> $o/bf16_c3.err || exit 3
for f in $o/c2_*.json $o/b*_*.json $o/c3_headline.json $o/bf16_c3.json; do python3 -c "
import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']
print('$f'.split('/')[-1], 'enc %.3f M sym/s' % (d['value']/1e6), 'ms/step %.4f' % d['ms_per_step'], 'dec', p.get('decode',{}).get('symbols_per_s'), 'oracle', p.get('bit_exact_vs_oracle'))"; done
