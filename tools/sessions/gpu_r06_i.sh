#!/bin/bash
# Round 6: (1) the lean step with per-iteration bounds (one CDF load per step): lean,
# drop-in, parity and flush tests; drop-in, c2 u32 / u64 lines.  (2) bf16 c3 row stats,
# slot permutation variants A/B.  (3) VERDICT r5 item 6: bench.py's c2 workload under
# rocprofv3 --pmc from saved inputs (no torch RNG kernel in the profiled process), then,
# last, the generating run itself under --pmc with python3 -X faulthandler (it crashed in
# torch.randn's launch in r06f: the frame is kept in profiles/r06/pmc_rng/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06i}; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_lean.py tests/test_gpu_dropin.py tests/test_gpu_parity.py tests/test_gpu_flush.py > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python3 tools/dropin_bench.py --out $o/dropin.json > $o/dropin.log 2>&1 || exit 3
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 5 --warmup 2 --decode-reps 3"
timeout -k 10 200 $C2 > $o/c2_1.json 2> $o/c2.err || exit 3
timeout -k 10 200 $C2 --pmf-bits 64 > $o/c2_u64.json 2> $o/c2_u64.err || exit 3
timeout -k 10 200 $C2 > $o/c2_2.json 2> $o/c2.err || exit 3
cat $o/dropin.json
for f in c2_1 c2_2 c2_u64; do python3 -c "
import json; d=json.loads([l for l in open('$o/$f.json') if l.startswith('{')][-1]); p=d['parity']
print('$f', '%.3f M sym/s' % (d['value']/1e6), 'dec %.3f M' % (p['decode']['symbols_per_s']/1e6), 'dec us/step %.3f' % (1e3*p['decode']['kernel_ms_per_step']), 'exact', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'))"; done
for v in perm perm_late; do
  LAC_LIB=tools/_probe/liblac_$v.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
      tests/test_gpu_logits.py -k "c3 or shape or bf16" > $o/t_$v.log 2>&1
  rc=$?; tail -1 $o/t_$v.log; [ $rc -eq 0 ] || exit 3
done
for i in 1 2; do
  timeout -k 10 120 python3 tools/q1_b2b.py --vocab 32000 --reps 20 > $o/q_base_$i.json 2>> $o/err.log || exit 3
  for v in perm perm_late; do
    LAC_LIB=tools/_probe/liblac_$v.so timeout -k 10 120 python3 tools/q1_b2b.py --vocab 32000 --reps 20 > $o/q_${v}_$i.json 2>> $o/err.log || exit 3
  done
done
for f in $o/q_*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); print('$f', {k: (round(v['q1_stats_ms_per_launch']*1e3/16, 2), round(v['frac_of_8TBps'], 4), v.get('q1_decode_us_per_step') and round(v['q1_decode_us_per_step'], 2)) for k, v in d.items() if isinstance(v, dict)})"; done
B="bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 3 --warmup 1 --decode-reps 1"
timeout -k 10 200 python3 $B --save-inputs /tmp/c2in > $o/save.json 2> $o/save.err || exit 3
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH" \
           "SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY"; do
  i=$(( ${i:-0} + 1 ))
  timeout -s KILL 180 rocprofv3 --pmc $set --kernel-trace -d $o/pmc$i -o run --output-format csv -- python3 $B --load-inputs /tmp/c2in > $o/pmc$i.json 2> $o/pmc$i.err
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || exit 3
done
tail -c 200 $o/pmc1.json
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU --kernel-trace -d $o/pmc_fh -o run --output-format csv -- python3 -X faulthandler $B > $o/pmc_fh.json 2> $o/pmc_fh.err
echo "faulthandler run rc=$?"
exit 0
