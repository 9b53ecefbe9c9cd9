#!/bin/bash
# Round 5: one-launch pack (k_pack) + the prefetching bf16 c3 decode form (shape 6 in
# decode, streamed butterfly): dist/logits/fuzz GPU tests, back-to-back row-stats
# timings AUTO (6) vs the old decode form (4), bf16 c3 bench lines, gather A/B + trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05c}; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py tests/test_gpu_logits.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/t.log 2>&1
rc=$?; tail -3 $o/t.log; [ $rc -eq 0 ] || exit 3
for r in 1 2; do
  timeout -k 10 200 python3 tools/q1_b2b.py --vocab 32000 --reps 10 > $o/b2b_auto$r.json 2> $o/b2b_auto$r.err || exit 3
  timeout -k 10 200 python3 tools/q1_b2b.py --vocab 32000 --reps 10 --q1-shape 4 > $o/b2b_s4_$r.json 2> $o/b2b_s4_$r.err || exit 3
  cat $o/b2b_auto$r.json $o/b2b_s4_$r.json
done
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --input logits-bf16 --steps 20 --warmup 3 --cpu-baseline off --decode-reps 5 > $o/bf16c3_$r.json 2> $o/bf16c3_$r.err || exit 3
  timeout -k 10 200 python3 bench.py --gather --steps 40 --warmup 5 --cpu-baseline off > $o/gather$r.json 2> $o/gather$r.err || exit 3
  timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --cpu-baseline off > $o/plain$r.json 2> $o/plain$r.err || exit 3
done
python3 tools/sessions/ab/summ.py $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/trace -o run --output-format csv -- python3 bench.py --gather --steps 20 --warmup 3 --cpu-baseline off > $o/trace.log 2>&1 || exit 3
