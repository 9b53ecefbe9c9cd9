#!/bin/bash
# Paired row stats (shape 19): logits GPU tests, then f32 bench lines (AUTO = 19 vs 14 / 10).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-pair}; mkdir -p $o
step() {
    local name=$1 secs=$2; shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "$o/$name.out" 2> "$o/$name.err"
    local rc=$?
    echo "== $name rc=$rc"; tail -n 2 "$o/$name.out" | cut -c1-400
    [ $rc -ne 0 ] && { tail -n 20 "$o/$name.err"; exit $rc; }
    return 0
}
B="python3 bench.py --cpu-baseline off --input logits-f32"
step tests_logits 400 python3 -u -m pytest tests/test_gpu_logits.py -q -x -rf --timeout 120 --timeout-method thread
step f32_c4_auto 200 $B --vocab 128256 --steps 5 --tokens 8
step f32_c4_sh14 200 $B --vocab 128256 --steps 5 --tokens 8 --q1-shape 14
step f32_c4_auto16 200 $B --vocab 128256 --steps 5 --tokens 16
step f32_v65540 200 $B --vocab 65540 --steps 5 --tokens 8
echo "== done"
