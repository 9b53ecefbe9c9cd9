#!/bin/bash
# Same-box A/B of build variants (tools/_probe/liblac_<v>.so; "cur" = the in-tree library):
# bf16 logits decode (k_q1_stats + k_q1_decode) at c3 and the c2 pmf decode.
# gpurun -- bash tools/sessions/ab/ab_r04_q1.sh <outdir> <variant>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/${1:-ab_q1}; shift; mkdir -p $o
VARS="${*:-cur pre}"
B="python3 bench.py --cpu-baseline off --steps 10 --warmup 5 --decode-reps 5 --input logits-bf16"
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 5 --warmup 2 --decode-reps 5"
run() {   # run <tag> <variant> <cmd...>
    local tag=$1 v=$2; shift 2
    local L=; [ $v != cur ] && L=tools/_probe/liblac_$v.so
    timeout -k 10 200 env ${L:+LAC_LIB=$L} "$@" > $o/${tag}_$v.json 2> $o/${tag}_$v.err || { tail -20 $o/${tag}_$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$o/${tag}_$v.json').read().strip().splitlines()[-1]); p=d['parity']['decode']; print('$tag $v', {k: round(1e3*x, 3) for k, x in p['kernel_ms_per_step_each'].items()}, 'rt', d['parity']['round_trip_all_streams'])"
}
for r in 1 2; do
    [ -n "${NO_C3:-}" ] || for v in $VARS; do run c3_$r $v $B; done
    for v in $VARS; do run c2_$r $v $C2; done
done
