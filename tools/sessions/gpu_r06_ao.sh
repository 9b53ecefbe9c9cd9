#!/bin/bash
# Round 6: a stream that leaves the lean step gets that step from k_decode_seq and the lean
# step again (three rounds per launch group): lean / drop-in
# / parity / api / fuzz tests, c2 u32 / u64 lines, one-stream V = 65536 u64 (2.6 us per step
# before: one row in 2048 can fudge, and the stream then finished its launch group on
# k_decode_seq), and the drop-in line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06ao}; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_lean.py tests/test_gpu_dropin.py tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_fuzz.py tests/test_gpu_flush.py > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || exit 3
C2="python3 bench.py --cpu-baseline off --streams 1 --steps 3 --warmup 1 --decode-reps 3"
timeout -k 10 200 $C2 --tokens 4096 > $o/c2_u32.json 2> $o/c2.err || exit 3
timeout -k 10 200 $C2 --tokens 4096 --pmf-bits 64 > $o/c2_u64.json 2> $o/c2.err || exit 3
timeout -k 10 200 $C2 --tokens 2048 --vocab 65536 --pmf-bits 64 > $o/v65536_u64.json 2> $o/c2.err || exit 3
timeout -k 10 300 python3 tools/dropin_bench.py --out $o/dropin.json > $o/dropin.log 2>&1 || exit 3
for f in $o/c2_u32.json $o/c2_u64.json $o/v65536_u64.json; do python3 -c "
import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']
print('$(basename $f)', 'dec us/step %.3f' % (1e3*p['decode']['kernel_ms_per_step']), 'exact', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'))"; done
python3 -c "import json; d=json.load(open('$o/dropin.json')); print('dropin decode', d['decode_sym_per_s'], d['decode_ok'])"
