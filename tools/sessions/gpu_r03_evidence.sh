#!/bin/bash
# Round 3 evidence for the wide row-stats shapes: rocprofv3 kernel stats and one
# FETCH_SIZE pass each (separate runs) of the AUTO logits bench at bf16 Qwen2
# (shape 22), bf16 262144 and f32 Qwen2 (shape 23).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-evidence}; mkdir -p $o
step() {   # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "== $name"
    timeout -s KILL "$secs" "$@" > "$o/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -n 1 "$o/$name.log" | cut -c1-200
    [ $rc -ne 0 ] && { tail -n 20 "$o/$name.log"; exit $rc; }
    return 0
}
B="python3 bench.py --cpu-baseline off"
for cfg in "bf16 151936 8" "bf16 262144 4" "f32 151936 4"; do
  set -- $cfg
  n=${1}_$2
  step stats_$n 300 rocprofv3 --kernel-trace --stats -d $o/stats_$n -o run --output-format csv -- $B --input logits-$1 --vocab $2 --tokens $3 --steps 10 --warmup 3
  step pmc_$n 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $o/pmc_$n -o run --output-format csv -- $B --input logits-$1 --vocab $2 --tokens $3 --steps 3 --warmup 1
done
echo "== done"
