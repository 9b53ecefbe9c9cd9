#!/bin/bash
# Round 6 evidence session (after the lean rounds): run of the committed library -- the whole GPU suite,
# smoke, the default bench (headline, cpu_baseline), its rocprofv3 kernel stats and one
# FETCH_SIZE pass (last), and the c2 (u32, u64), bf16 c3, gather (world 1), gloo world-2 and
# drop-in lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06final5}; mkdir -p $o
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/gpu_tests.log 2>&1
rc=$?; tail -3 $o/gpu_tests.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 3
tail -1 $o/smoke.log
timeout -k 10 300 python3 bench.py > $o/bench_c3.json 2> $o/bench_c3.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run --output-format csv -- python3 bench.py --cpu-baseline off > $o/stats_pmf.json 2> $o/prof.log || exit 3
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 5 --warmup 2 --decode-reps 3"
timeout -k 10 200 $C2 > $o/c2.json 2> $o/c2.err || exit 3
timeout -k 10 200 $C2 --pmf-bits 64 > $o/c2_u64.json 2> $o/c2_u64.err || exit 3
timeout -k 10 300 python3 bench.py --input logits-bf16 --cpu-baseline off --decode-reps 20 > $o/bf16_c3.json 2> $o/bf16_c3.err || exit 3
timeout -k 10 300 python3 bench.py --gather --cpu-baseline off > $o/gather_w1.json 2> $o/gather_w1.err || exit 3
LAC_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 > $o/gloo2.json 2> $o/gloo2.err || exit 3
timeout -k 10 300 python3 tools/dropin_bench.py --out $o/dropin.json > $o/dropin.log 2>&1 || exit 3
# last: the one counter pass (one FETCH_SIZE counter, as round 5's two passes)
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $o/pmc -o run --output-format csv -- python3 bench.py --cpu-baseline off --steps 10 --warmup 2 --decode-reps 2 > $o/pmc_pmf.json 2> $o/pmc.log || exit 3
for f in bench_c3 stats_pmf c2 c2_u64 bf16_c3 gather_w1 gloo2; do python3 -c "
import json; d=json.loads([l for l in open('$o/$f.json') if l.startswith('{')][-1]); p=d['parity']; r=d['roofline']
print('$f', 'n_gpus', d['n_gpus'], '%.3f M sym/s' % (d['value']/1e6), 'ms/step %.4f' % d['ms_per_step'], 'frac', r.get('frac') and round(r['frac'],4), 'dec %.3f M' % (p['decode']['symbols_per_s']/1e6), 'exact', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'), 'gather_ok', p.get('gather_ok'), 'cpu', d.get('cpu_baseline') and round(d['cpu_baseline']['value']))"; done
grep -h "k_encode_fused" $o/prof/*kernel_stats.csv | head -2
python3 tools/pmc_summary.py $o/pmc k_encode_fused
tail -c 400 $o/dropin.json
