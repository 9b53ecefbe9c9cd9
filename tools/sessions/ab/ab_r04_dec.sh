#!/bin/bash
# Round 4 same-box A/B of the decode changes: round-start library (tools/_probe/liblac_base.so,
# built from the round's first commit) vs this tree's liblac.so; bf16 logits decode at
# c3 / c4 / Qwen2 / Llama-4 / o200k (the new library with AUTO and with shape 22 forced
# where AUTO keeps the slot forms), and the c2 pmf decode.  gpurun -- bash tools/sessions/ab/ab_r04_dec.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-ab_r04_dec}; mkdir -p $o
B="python3 bench.py --cpu-baseline off --steps 8 --warmup 5 --decode-reps 5 --input logits-bf16 --tokens 16"
for rep in 1 2; do
  for V in 32000 128256 151936 202048 200024; do
    timeout -k 10 300 env LAC_LIB=tools/_probe/liblac_base.so $B --vocab $V > $o/bf16_${V}_base_$rep.json 2> $o/err_${V}_base_$rep.txt || exit 3
    timeout -k 10 300 $B --vocab $V > $o/bf16_${V}_new_$rep.json 2> $o/err_${V}_new_$rep.txt || exit 3
    if [ $V -gt 163840 ]; then
      timeout -k 10 300 $B --vocab $V --q1-shape 22 > $o/bf16_${V}_new22_$rep.json 2> $o/err_${V}_new22_$rep.txt || exit 3
    fi
  done
  C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 2 --warmup 1 --decode-reps 3"
  timeout -k 10 300 env LAC_LIB=tools/_probe/liblac_base.so $C2 > $o/c2_base_$rep.json 2> $o/err_c2_base_$rep.txt || exit 3
  timeout -k 10 300 $C2 > $o/c2_new_$rep.json 2> $o/err_c2_new_$rep.txt || exit 3
done
python3 tools/sessions/ab/summ.py $o
