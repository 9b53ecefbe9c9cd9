#!/bin/bash
# Round 3: full GPU suite + smoke on the current library, the headline bench, the
# AUTO logits lines the wide shapes changed, and the u64 decode PMC pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-check}; mkdir -p $o
step() {   # step <name> <seconds> <cmd...>: any failure ends the session
    local name=$1 secs=$2; shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "$o/$name.json" 2> "$o/$name.err"
    local rc=$?
    echo "== $name rc=$rc"; tail -n 2 "$o/$name.json" | cut -c1-300
    [ $rc -ne 0 ] && { tail -n 30 "$o/$name.err"; exit $rc; }
    return 0
}
step tests 900 python3 -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench_c3 300 python3 bench.py
B="python3 bench.py --cpu-baseline off --steps 10 --warmup 5"
step auto_bf16_262144 200 $B --input logits-bf16 --vocab 262144 --tokens 4
step auto_f32_151936 200 $B --input logits-f32 --vocab 151936 --tokens 4
step auto_f32_65540 200 $B --input logits-f32 --vocab 65540 --tokens 8
step auto_bf16_c4 200 $B --input logits-bf16 --vocab 128256 --tokens 8
step auto_bf16_c3 200 $B --input logits-bf16
bash tools/sessions/gpu_r03_u64pmc.sh $(basename $o)/u64pmc || exit 3
echo "== done"
