#!/bin/bash
# k_q1_decode per-step time against the stream count (bf16 c3 rows): latency- or issue-bound?
# gpurun -- bash tools/sessions/ab/ab_r04_q1streams.sh <outdir>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/${1:-q1streams}; mkdir -p $o
for B in 256 1024 2048 4096 8192; do
    timeout -k 10 200 python3 bench.py --cpu-baseline off --steps 5 --warmup 3 --decode-reps 5 --input logits-bf16 --streams $B > $o/b$B.json 2> $o/b$B.err || { tail -20 $o/b$B.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$o/b$B.json').read().strip().splitlines()[-1]); p=d['parity']['decode']; print('B=$B', {k: round(1e3*x, 3) for k, x in p['kernel_ms_per_step_each'].items()}, 'rt', d['parity']['round_trip_all_streams'])"
done
