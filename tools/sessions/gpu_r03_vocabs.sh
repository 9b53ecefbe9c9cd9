#!/bin/bash
# Round 3: logits row stats at the 100k-200k vocabularies past shape 22's 20480
# vectors (Llama-4 202048 / o200k 200024 in bf16, cl100k 100280 / DeepSeek 102400 in
# f32): AUTO and the forced group forms, same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-vocabs}; mkdir -p $o
B="python3 bench.py --cpu-baseline off --steps 10 --warmup 5 --tokens 4"
for cfg in "bf16 202048" "bf16 200024" "f32 100280" "f32 102400" "bf16 100280"; do
  set -- $cfg
  for sh in 0 19 21 23; do
    timeout -k 10 200 $B --input logits-$1 --vocab $2 --q1-shape $sh > $o/${1}_${2}_s$sh.json 2> $o/${1}_${2}_s$sh.err || exit 3
  done
  echo "$cfg ok"
done
python3 tools/sessions/ab/summ.py $o
