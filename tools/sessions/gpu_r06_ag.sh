#!/bin/bash
# Round 6: two chunk bounds per lane for u32 rows too (tools/_probe/liblac_cw32.so: 128 chunks,
# one CDF load per step at V=32000) against the kept one bound: lean tests on the variant,
# then c2 u32 decode and the static-row probe, A/B twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06ag}; mkdir -p $o
LAC_LIB=tools/_probe/liblac_cw32.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_lean.py tests/test_gpu_dropin.py > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || exit 3
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 3 --warmup 1 --decode-reps 3"
P="python3 tools/dec_phase_probe.py --tokens 4096 --static"
for rep in 1 2; do
for v in default cw32; do
    if [ $v = default ]; then L=""; else L=tools/_probe/liblac_$v.so; fi
    LAC_LIB=$L timeout -k 10 200 $C2 > $o/${v}_u32_$rep.json 2> $o/${v}.err || exit 3
    LAC_LIB=$L timeout -k 10 200 $P > $o/${v}_static_$rep.txt 2>> $o/${v}.err || exit 3
done
done
for f in $o/*_u32_*.json; do python3 -c "
import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']
print('$(basename $f)', 'dec us/step %.3f' % (1e3*p['decode']['kernel_ms_per_step']), 'exact', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'))"; done
for f in $o/*_static_*.txt; do echo "$(basename $f) $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["kernel_us_per_step"], d["round_trip"])' $f)"; done
