#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
o=gpurun_out/pair_bf16; mkdir -p $o
step() {
    local name=$1 secs=$2; shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "$o/$name.out" 2> "$o/$name.err"
    local rc=$?
    echo "== $name rc=$rc"; tail -n 1 "$o/$name.out" | cut -c1-200
    [ $rc -ne 0 ] && { tail -n 20 "$o/$name.err"; exit $rc; }
    return 0
}
B="python3 bench.py --cpu-baseline off --input logits-bf16 --steps 5"
step tests_logits 400 python3 -u -m pytest tests/test_gpu_logits.py -q -x -rf --timeout 120 --timeout-method thread
step bf16_256k_auto 200 $B --vocab 256000 --tokens 8
step bf16_256k_19 200 $B --vocab 256000 --tokens 8 --q1-shape 19
step bf16_262k_auto 200 $B --vocab 262144 --tokens 8
step bf16_262k_19 200 $B --vocab 262144 --tokens 8 --q1-shape 19
step f32_c4_auto 200 python3 bench.py --cpu-baseline off --input logits-f32 --steps 5 --vocab 128256 --tokens 8
step bf16_c4 200 $B --vocab 128256
step bf16_c3 200 $B --vocab 32000 --steps 20
echo "== done"
