#!/bin/bash
# c2 decode: decode GPU tests, the lean kernel's phase split (probe build), the product
# line and the k_decode_seq-only build (LAC_LEAN=0).  gpurun -- bash tools/sessions/ab/ab_r04_lean_phases.sh [outdir]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/${1:-lean_phases}; mkdir -p $o
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_lean.py tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_checkpoint.py tests/test_gpu_api.py tests/test_gpu_flush.py -m gpu -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
if [ -f tools/_probe/liblac_phases.so ]; then
timeout -k 10 200 env LAC_LIB=tools/_probe/liblac_phases.so python3 tools/dec_phase_probe.py --kernel lean > $o/phases.json 2> $o/phases.err || { tail -20 $o/phases.err; exit 1; }
cat $o/phases.json
fi
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 5 --warmup 2 --decode-reps 5"
for v in lean nohelp seq lean2 nohelp2; do
    case $v in seq) L=tools/_probe/liblac_nolean.so;; nohelp*) L=tools/_probe/liblac_nohelp.so;; *) L=;; esac
    timeout -k 10 200 env ${L:+LAC_LIB=$L} $C2 > $o/c2_$v.json 2> $o/c2_$v.err || { tail -20 $o/c2_$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$o/c2_$v.json').read().strip().splitlines()[-1]); p=d['parity']; print('$v c2 dec us/step', round(1e3*p['decode']['kernel_ms_per_step'], 4), 'rt', p['round_trip_all_streams'], 'exact', p['bit_exact_vs_oracle'])"
done
B="python3 bench.py --cpu-baseline off --steps 10 --warmup 5 --decode-reps 5 --input logits-bf16"
for v in c3 c4; do
    if [ $v = c4 ]; then X="--vocab 128256"; else X=; fi
    timeout -k 10 200 $B $X > $o/bf16_$v.json 2> $o/bf16_$v.err || { tail -20 $o/bf16_$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$o/bf16_$v.json').read().strip().splitlines()[-1]); p=d['parity']['decode']; print('bf16 $v', {k: round(1e3*x, 3) for k, x in p['kernel_ms_per_step_each'].items()}, 'rt', d['parity']['round_trip_all_streams'])"
done
