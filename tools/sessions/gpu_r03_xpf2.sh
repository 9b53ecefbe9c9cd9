#!/bin/bash
# Round 3: fine decoder with two groups in flight (LAC_DEC_XPF=2 variant) vs one,
# same box: c3 u32 and llama-scale u64 decode.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-xpf2}; mkdir -p $o
B="python3 bench.py --cpu-baseline off --steps 5 --warmup 2 --decode-reps 5"
for rep in 1 2; do
  for v in one two; do
    lib=lac_amd/liblac.so; [ $v = two ] && lib=tools/sessions/ab/liblac_r03_xpf2.so
    LAC_LIB=$lib timeout -k 10 300 $B > $o/u32_${v}_$rep.json 2> $o/u32_${v}_$rep.err || exit 3
    LAC_LIB=$lib timeout -k 10 300 $B --pmf-bits 64 > $o/u64_${v}_$rep.json 2> $o/u64_${v}_$rep.err || exit 3
    echo "$v $rep ok"
  done
done
python3 tools/sessions/ab/summ.py $o
