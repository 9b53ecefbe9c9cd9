#!/bin/bash
# Row groups of 2..4 blocks (shape 19): logits GPU tests, then bench lines at Qwen2 / Gemma vocabularies.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
o=gpurun_out/${1:-groups}; mkdir -p $o
step() {
    local name=$1 secs=$2; shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "$o/$name.out" 2> "$o/$name.err"
    local rc=$?
    echo "== $name rc=$rc"; tail -n 1 "$o/$name.out" | cut -c1-160
    [ $rc -ne 0 ] && { tail -n 20 "$o/$name.err"; exit $rc; }
    return 0
}
B="python3 bench.py --cpu-baseline off --steps 5 --warmup 5"
step tests_logits 500 python3 -u -m pytest tests/test_gpu_logits.py -q -x -rf --timeout 120 --timeout-method thread
for cfg in "f32_152k:--input logits-f32 --vocab 151936 --tokens 8" "f32_152k_14:--input logits-f32 --vocab 151936 --tokens 8 --q1-shape 14" \
           "bf16_152k:--input logits-bf16 --vocab 151936 --tokens 8" "bf16_152k_8:--input logits-bf16 --vocab 151936 --tokens 8 --q1-shape 8" \
           "bf16_262k:--input logits-bf16 --vocab 262144 --tokens 8" "f32_256k:--input logits-f32 --vocab 256000 --tokens 4" \
           "f32_262k:--input logits-f32 --vocab 262144 --tokens 4" "f32_c4:--input logits-f32 --vocab 128256 --tokens 8"; do
  step ${cfg%%:*} 200 $B ${cfg#*:}
done
echo "== done"
