#!/bin/bash
# k_q1_decode table replication A/B (+ the logits GPU tests on the in-tree library).
# gpurun -- bash tools/sessions/ab/ab_r04_q1rep.sh <outdir> <variant>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/${1:-ab_q1rep}; shift; mkdir -p $o
VARS="${*:-cur rep1}"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_logits.py -m gpu -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
B="python3 bench.py --cpu-baseline off --steps 10 --warmup 5 --decode-reps 5 --input logits-bf16"
run() {
    local tag=$1 v=$2; shift 2
    local L=; [ $v != cur ] && L=tools/_probe/liblac_$v.so
    timeout -k 10 200 env ${L:+LAC_LIB=$L} "$@" > $o/${tag}_$v.json 2> $o/${tag}_$v.err || { tail -20 $o/${tag}_$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$o/${tag}_$v.json').read().strip().splitlines()[-1]); p=d['parity']['decode']; print('$tag $v', {k: round(1e3*x, 3) for k, x in p['kernel_ms_per_step_each'].items()}, 'rt', d['parity']['round_trip_all_streams'])"
}
for r in 1 2; do
    for v in $VARS; do run c3_$r $v $B; done
    for v in $VARS; do run c4_$r $v $B --vocab 128256; done
done
