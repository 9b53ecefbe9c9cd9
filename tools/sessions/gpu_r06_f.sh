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
