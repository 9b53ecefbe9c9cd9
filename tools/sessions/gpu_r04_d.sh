#!/bin/bash
# Round 4: logits GPU tests on the spill-free wide decode form, back-to-back row-stats
# timings (encode vs decode form), stats-path decode at 1..1024 streams old vs new.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r04d}; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_logits.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || exit 3
for V in 151936 202048 32000 128256; do
  timeout -k 10 300 python3 tools/q1_b2b.py --vocab $V > $o/b2b_$V.json 2> $o/b2b_$V.err || exit 3
  cat $o/b2b_$V.json
done
for Bn in 1 64 256 1024; do
  T=$(( Bn == 1 ? 2048 : 64 ))
  for lib in base new; do
    if [ $lib = base ]; then L="env LAC_LIB=tools/_probe/liblac_base.so"; else L=""; fi
    timeout -k 10 300 $L python3 bench.py --cpu-baseline off --streams $Bn --tokens $T --steps 2 --warmup 1 --decode-reps 3 > $o/stats_${Bn}_$lib.json 2> $o/stats_${Bn}_$lib.err || exit 3
  done
done
python3 tools/sessions/ab/summ.py $o
