#!/bin/bash
# Round 3: shape 22 with its rolling prefetch -- parity tests, then same-box A/B
# against AUTO (row groups) at bf16 Qwen2 / 131080 and f32 65540.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-wide2}; mkdir -p $o
step() {   # step <name> <seconds> <cmd...>: any failure ends the session
    local name=$1 secs=$2; shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "$o/$name.json" 2> "$o/$name.err"
    local rc=$?
    echo "== $name rc=$rc"; tail -n 3 "$o/$name.json" | cut -c1-300
    [ $rc -ne 0 ] && { tail -n 30 "$o/$name.err"; exit $rc; }
    return 0
}
step tests 600 python3 -u -m pytest tests/test_gpu_logits.py -x -q -rf --timeout 300 --timeout-method thread -k "every_q1_shape or paired_row_stats or option_range"
B="python3 bench.py --cpu-baseline off --steps 10 --warmup 5"
for rep in 1 2; do
  for sh in 0 22; do
    step bf16_151936_s${sh}_$rep 200 $B --input logits-bf16 --vocab 151936 --tokens 8 --q1-shape $sh
    step bf16_131080_s${sh}_$rep 200 $B --input logits-bf16 --vocab 131080 --tokens 8 --q1-shape $sh
    step f32_65540_s${sh}_$rep 200 $B --input logits-f32 --vocab 65540 --tokens 8 --q1-shape $sh
  done
done
python3 tools/sessions/ab/summ.py $o
echo "== done"
