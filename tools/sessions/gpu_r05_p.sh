#!/bin/bash
# Round 5: bench.py's gather check (gather_ok) after the fix that compares each stream
# over its own bytes only: world 1 over RCCL (--gather), then bench.py's launcher with
# gloo ranks sharing the one GPU: c3 on 2 and 4 ranks, the c5 shape on 8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05p}; mkdir -p $o
timeout -k 10 300 python3 bench.py --gather --steps 20 --warmup 3 --cpu-baseline off > $o/c3_gather_w1.txt 2> $o/c3_gather_w1.err || exit 3
tail -n1 $o/c3_gather_w1.txt | cut -c1-300
LAC_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 10 --warmup 2 --cpu-baseline off --decode-reps 2 > $o/c3_gloo2.txt 2> $o/c3_gloo2.err || exit 3
LAC_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 4 --steps 5 --warmup 1 --cpu-baseline off --decode-reps 2 > $o/c3_gloo4.txt 2> $o/c3_gloo4.err || exit 3
LAC_DIST_BACKEND=gloo timeout -k 10 600 python3 bench.py --gpus 8 --vocab 128256 --tokens 4 --steps 2 --warmup 1 --cpu-baseline off --decode-reps 1 > $o/c5_gloo8.txt 2> $o/c5_gloo8.err || exit 3
for f in c3_gather_w1 c3_gloo2 c3_gloo4 c5_gloo8; do
  python3 -c "import json,sys; j=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], j['n_gpus'], j['value'], 'gather_ok', j['parity'].get('gather_ok'), 'oracle', j['parity'].get('bit_exact_vs_oracle'))" $o/$f.txt
done
