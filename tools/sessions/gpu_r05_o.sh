#!/bin/bash
# Round 5: multi-rank rehearsals of bench.py's own launcher on the one-GPU box (gloo,
# ranks sharing the GPU): the c5 shape on 8 ranks (V=128256, 4096 streams per rank; 4
# symbols per stream per job to fit 8 ranks' tables in one GPU's HBM) and c3 on 4 ranks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05o}; mkdir -p $o
LAC_DIST_BACKEND=gloo timeout -k 10 600 python3 bench.py --gpus 8 --vocab 128256 --tokens 4 --steps 2 --warmup 1 --cpu-baseline off --decode-reps 1 > $o/c5_gloo8.txt 2> $o/c5_gloo8.err || exit 3
tail -n1 $o/c5_gloo8.txt | cut -c1-600
LAC_DIST_BACKEND=gloo timeout -k 10 600 python3 bench.py --gpus 4 --steps 5 --warmup 1 --decode-reps 2 > $o/c3_gloo4.txt 2> $o/c3_gloo4.err || exit 3
tail -n1 $o/c3_gloo4.txt | cut -c1-600
