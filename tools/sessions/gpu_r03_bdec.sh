#!/bin/bash
# Round 3: bf16 decode row stats of 20481..26112-vector rows in shape 22 (36 register
# vectors + 15 LDS slots, 16 table copies) vs AUTO's slot forms -- logits tests, then
# the decode stats of bf16 202048 / 200024 both ways, same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-bdec}; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_logits.py -x -q -rf --timeout 300 --timeout-method thread -k "every_q1_shape or paired_row_stats" > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 3; }
tail -2 $o/tests.log
B="python3 bench.py --cpu-baseline off --steps 10 --warmup 5 --tokens 4 --decode-reps 5"
for rep in 1 2; do
  for V in 202048 200024; do
    for sh in 0 22; do
      timeout -k 10 200 $B --input logits-bf16 --vocab $V --q1-shape $sh > $o/bf16_${V}_s${sh}_$rep.json 2> $o/bf16_${V}_s${sh}_$rep.err || exit 3
    done
  done
done
python3 tools/sessions/ab/summ.py $o
