#!/bin/bash
# Row groups with two rows per block (shape 20) vs one (19): logits tests, fuzz, bench lines.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
o=gpurun_out/${1:-groups2}; mkdir -p $o
step() {
    local name=$1 secs=$2; shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "$o/$name.out" 2> "$o/$name.err"
    local rc=$?
    echo "== $name rc=$rc"; tail -n 1 "$o/$name.out" | cut -c1-120
    [ $rc -ne 0 ] && { tail -n 20 "$o/$name.err"; exit $rc; }
    return 0
}
step tests_logits 500 python3 -u -m pytest tests/test_gpu_logits.py tests/test_gpu_fuzz.py -q -x -rf --timeout 120 --timeout-method thread
B="python3 bench.py --cpu-baseline off --steps 5 --warmup 5 --tokens 8"
for cfg in "bf16_152k_19:--input logits-bf16 --vocab 151936 --q1-shape 19" "bf16_152k_20:--input logits-bf16 --vocab 151936 --q1-shape 20" \
           "bf16_131k_19:--input logits-bf16 --vocab 131080 --q1-shape 19" "bf16_131k_20:--input logits-bf16 --vocab 131080 --q1-shape 20" \
           "f32_65540_19:--input logits-f32 --vocab 65540 --q1-shape 19" "f32_65540_20:--input logits-f32 --vocab 65540 --q1-shape 20" \
           "f32_100k_19:--input logits-f32 --vocab 100000 --q1-shape 19" "f32_100k_20:--input logits-f32 --vocab 100000 --q1-shape 20" \
           "bf16_200k_19:--input logits-bf16 --vocab 200000 --q1-shape 19" "bf16_200k_20:--input logits-bf16 --vocab 200000 --q1-shape 20"; do
  step ${cfg%%:*} 200 $B ${cfg#*:}
done
echo "== done"
