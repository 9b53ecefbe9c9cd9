#!/bin/bash
# Round 6: u64 lean rows with two chunk bounds per lane (128 chunks: two loads per lane at
# V=32000 instead of four): lean and parity tests, c2 u32 / u64 lines twice, the static-row
# probe and the drop-in line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06af}; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_lean.py tests/test_gpu_dropin.py tests/test_gpu_parity.py > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || exit 3
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 3 --warmup 1 --decode-reps 3"
for rep in 1 2; do
    timeout -k 10 200 $C2 > $o/c2_u32_$rep.json 2> $o/c2.err || exit 3
    timeout -k 10 200 $C2 --pmf-bits 64 > $o/c2_u64_$rep.json 2> $o/c2.err || exit 3
done
P="python3 tools/dec_phase_probe.py --tokens 4096"
timeout -k 10 200 $P --static > $o/u32_static.json 2>> $o/err.log || exit 3
timeout -k 10 200 $P --pmf-bits 64 --static > $o/u64_static.json 2>> $o/err.log || exit 3
timeout -k 10 300 python3 tools/dropin_bench.py --out $o/dropin.json > $o/dropin.log 2>&1 || exit 3
for f in $o/c2_*.json; do python3 -c "
import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']
print('$(basename $f)', 'dec us/step %.3f' % (1e3*p['decode']['kernel_ms_per_step']), 'exact', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'))"; done
for f in $o/u*_static.json; do echo "$(basename $f) $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["kernel_us_per_step"], d["round_trip"])' $f)"; done
python3 -c "import json; d=json.load(open('$o/dropin.json')); print('dropin decode', d['decode_sym_per_s'], d['decode_ok'])"
