#!/bin/bash
# Round 3: shape 22 with LDS slots (rows of 20481..26112 vectors) -- logits parity
# tests, then AUTO vs the slot forms at Llama-4 / o200k (bf16) and cl100k / DeepSeek
# (f32) vocabularies, and the shape-23 rule's cases.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-vocabs2}; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_logits.py tests/test_gpu_fuzz.py -x -q -rf --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 3; }
tail -2 $o/tests.log
B="python3 bench.py --cpu-baseline off --steps 10 --warmup 5 --tokens 4"
for cfg in "bf16 202048" "bf16 200024" "f32 100280" "f32 102400"; do
  set -- $cfg
  for sh in 0 19; do
    timeout -k 10 200 $B --input logits-$1 --vocab $2 --q1-shape $sh > $o/${1}_${2}_s$sh.json 2> $o/${1}_${2}_s$sh.err || exit 3
  done
  echo "$cfg ok"
done
for cfg in "bf16 262144" "f32 151936" "bf16 151936"; do
  set -- $cfg
  timeout -k 10 200 $B --input logits-$1 --vocab $2 > $o/${1}_${2}_auto.json 2> $o/${1}_${2}_auto.err || exit 3
done
python3 tools/sessions/ab/summ.py $o
