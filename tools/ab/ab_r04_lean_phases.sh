#!/bin/bash
# c2 decode: decode GPU tests, the lean kernel's phase split (probe build), the product
# line and the k_decode_seq-only build (LAC_LEAN=0).  gpurun -- bash tools/ab/ab_r04_lean_phases.sh [outdir]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/${1:-lean_phases}; mkdir -p $o
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_lean.py tests/test_gpu_parity.py tests/test_gpu_checkpoint.py tests/test_gpu_api.py tests/test_gpu_flush.py -m gpu -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 200 env LAC_LIB=tools/_probe/liblac_phases.so python3 tools/dec_phase_probe.py --kernel lean > $o/phases.json 2> $o/phases.err || { tail -20 $o/phases.err; exit 1; }
cat $o/phases.json
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 5 --warmup 2 --decode-reps 5"
for v in lean seq noprod lean2 noprod2; do
    case $v in seq) L=tools/_probe/liblac_nolean.so;; noprod*) L=tools/_probe/liblac_noprod.so;; *) L=;; esac
    timeout -k 10 200 env ${L:+LAC_LIB=$L} $C2 > $o/c2_$v.json 2> $o/c2_$v.err || { tail -20 $o/c2_$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$o/c2_$v.json').read().strip().splitlines()[-1]); p=d['parity']; print('$v c2 dec us/step', round(1e3*p['decode']['kernel_ms_per_step'], 4), 'rt', p['round_trip_all_streams'], 'exact', p['bit_exact_vs_oracle'])"
done
