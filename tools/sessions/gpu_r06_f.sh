#!/bin/bash
# Round 6: (1) the coder's per-position cost in the ROCm serving loop:
# tools/serving_bench.py at B = 1 and 4096, V = 32000 bf16, tiny and small models, and a
# rocprofv3 kernel trace of each B for the per-kernel split; (2) bench.py's own c2
# workload under rocprofv3 --pmc (its tables now come from one
# reseeded generator).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06f}; mkdir -p $o
S="python3 tools/serving_bench.py"
timeout -k 10 300 $S --streams 1 --positions 256 --model tiny --out $o/b1_tiny.json > $o/b1_tiny.log 2>&1 || exit 3
timeout -k 10 300 $S --streams 1 --positions 256 --model small --out $o/b1_small.json > $o/b1_small.log 2>&1 || exit 3
timeout -k 10 600 $S --streams 4096 --positions 32 --model tiny --out $o/b4096_tiny.json > $o/b4096_tiny.log 2>&1 || exit 3
timeout -k 10 600 $S --streams 4096 --positions 32 --model small --out $o/b4096_small.json > $o/b4096_small.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/trace_b1 -o run --output-format csv -- python3 tools/serving_bench.py --streams 1 --positions 256 --model tiny > $o/trace_b1.log 2>&1 || exit 3
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $o/trace_b4096 -o run --output-format csv -- python3 tools/serving_bench.py --streams 4096 --positions 32 --model tiny > $o/trace_b4096.log 2>&1 || exit 3
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH --kernel-trace -d $o/pmc_c2 -o run --output-format csv -- python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 3 --warmup 1 --decode-reps 1 > $o/pmc_c2.json 2> $o/pmc_c2.err || exit 3
cat $o/b1_tiny.json $o/b1_small.json $o/b4096_tiny.json $o/b4096_small.json
tail -c 300 $o/pmc_c2.json
# bf16 c3 logits row statistics, slot permutation (PERM: the streamed butterfly's rolling
# prefetch in address order), alone and with the late tail, A/B against the default
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
