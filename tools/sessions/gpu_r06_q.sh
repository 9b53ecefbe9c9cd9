#!/bin/bash
# Round 6: the next launch group's statistics by worker workgroups of the lean launch (fewer than
# 8 streams), first group of 256 steps: lean tests, c2 u32 / u64 lines, and a kernel trace of
# stats pass's share of a decode step).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06q}; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_lean.py tests/test_gpu_dropin.py tests/test_gpu_parity.py tests/test_gpu_api.py > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || exit 3
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 5 --warmup 2 --decode-reps 3"
timeout -k 10 200 $C2 > $o/c2_1.json 2> $o/c2.err || exit 3
timeout -k 10 200 $C2 --pmf-bits 64 > $o/c2_u64.json 2> $o/c2_u64.err || exit 3
timeout -k 10 200 $C2 > $o/c2_2.json 2> $o/c2.err || exit 3
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/tr32 -o run --output-format csv -- $C2 > $o/tr32.json 2> $o/tr32.log || exit 3
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/tr64 -o run --output-format csv -- $C2 --pmf-bits 64 > $o/tr64.json 2> $o/tr64.log || exit 3
for f in c2_1 c2_2 c2_u64; do python3 -c "
import json; d=json.loads([l for l in open('$o/$f.json') if l.startswith('{')][-1]); p=d['parity']
print('$f', '%.3f M sym/s' % (d['value']/1e6), 'dec %.3f M' % (p['decode']['symbols_per_s']/1e6), 'dec us/step %.3f' % (1e3*p['decode']['kernel_ms_per_step']), 'exact', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'))"; done
for t in tr32 tr64; do cp /tmp/$t/run_kernel_stats.csv $o/${t}_kernel_stats.csv; grep -h "k_dec_stats\|k_decode_lean\|k_decode_seq\|k_lean_window" $o/${t}_kernel_stats.csv | cut -c1-60,200-400 || true; done
# (the traces themselves stay in /tmp: every torch kernel of the synthetic tables is in them, > 64 MiB)
