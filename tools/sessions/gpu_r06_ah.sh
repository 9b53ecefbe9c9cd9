#!/bin/bash
# Round 6: k_q1_decode issuing the next row's chunk-total prefetch after the step's group
# loads (unconditional, buffers padded a row) instead of before them: logits tests, then the
# bf16 c3 back-to-back row stats + k_q1_decode times A/B against the old order
# (tools/_probe/liblac_pf0.so), twice, and the bf16 c3 bench line of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06ah}; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_logits.py tests/test_gpu_fuzz.py > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || exit 3
for rep in 1 2; do
for v in default pf0; do
    if [ $v = default ]; then L=""; else L=tools/_probe/liblac_$v.so; fi
    LAC_LIB=$L timeout -k 10 300 python3 tools/q1_b2b.py --vocab 32000 --reps 20 > $o/${v}_b2b_$rep.json 2> $o/${v}.err || exit 3
done
done
for v in default pf0; do
    if [ $v = default ]; then L=""; else L=tools/_probe/liblac_$v.so; fi
    LAC_LIB=$L timeout -k 10 300 python3 bench.py --input logits-bf16 --cpu-baseline off --decode-reps 20 > $o/${v}_bf16.json 2> $o/${v}_bf16.err || exit 3
done
for f in $o/*_b2b_*.json; do echo "$(basename $f) $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print({k: v for k, v in d.items() if "decode" in k})' $f)"; done
for f in $o/*_bf16.json; do python3 -c "
import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']['decode']
print('$(basename $f)', 'dec %.2f M sym/s' % (p['symbols_per_s']/1e6), p.get('kernel_ms_per_step_each'), 'exact', d['parity'].get('bit_exact_vs_oracle'))"; done
