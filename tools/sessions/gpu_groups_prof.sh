#!/bin/bash
# rocprofv3 kernel stats + FETCH_SIZE passes (separate runs) of the row-group shapes: f32 Qwen2 (K = 3), f32 256000 (K = 4).
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
o=gpurun_out/groups_prof; mkdir -p $o
B="python3 bench.py --cpu-baseline off --input logits-f32"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof_qwen -o run --output-format csv -- $B --vocab 151936 --tokens 8 --steps 5 --warmup 3 > $o/stats_qwen.out 2>$o/stats_qwen.err || exit 3
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $o/pmc_qwen -o run --output-format csv -- $B --vocab 151936 --tokens 8 --steps 3 --warmup 1 > $o/pmc_qwen.out 2>$o/pmc_qwen.err || exit 3
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $o/pmc_256k -o run --output-format csv -- $B --vocab 256000 --tokens 4 --steps 3 --warmup 1 > $o/pmc_256k.out 2>$o/pmc_256k.err || exit 3
echo done
