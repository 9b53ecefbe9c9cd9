#!/bin/bash
# Round 3: shape 22 (AUTO for 16385..20480-vector rows) -- logits parity tests, then
# same-box A/B against the register + slot shape 15 on rows it holds (<= 16384 vectors).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-wide3}; mkdir -p $o
step() {   # step <name> <seconds> <cmd...>: any failure ends the session
    local name=$1 secs=$2; shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "$o/$name.json" 2> "$o/$name.err"
    local rc=$?
    echo "== $name rc=$rc"; tail -n 2 "$o/$name.json" | cut -c1-200
    [ $rc -ne 0 ] && { tail -n 30 "$o/$name.err"; exit $rc; }
    return 0
}
step tests 900 python3 -u -m pytest tests/test_gpu_logits.py tests/test_gpu_fuzz.py -x -q -rf --timeout 300 --timeout-method thread
B="python3 bench.py --cpu-baseline off --steps 10 --warmup 5"
for rep in 1 2; do
  step auto_bf16_151936_$rep 200 $B --input logits-bf16 --vocab 151936 --tokens 8
  step auto_bf16_131080_$rep 200 $B --input logits-bf16 --vocab 131080 --tokens 8
  for sh in 0 22; do
    step bf16_128256_s${sh}_$rep 200 $B --input logits-bf16 --vocab 128256 --tokens 8 --q1-shape $sh
    step f32_65536_s${sh}_$rep 200 $B --input logits-f32 --vocab 65536 --tokens 8 --q1-shape $sh
    step bf16_100000_s${sh}_$rep 200 $B --input logits-bf16 --vocab 100000 --tokens 8 --q1-shape $sh
  done
done
# shape 23 (wide row groups) vs AUTO (row slots) on rows past 20480 vectors
for rep in 1 2; do
  for sh in 0 23; do
    step bf16_262144_s${sh}_$rep 200 $B --input logits-bf16 --vocab 262144 --tokens 4 --q1-shape $sh
    step bf16_256000_s${sh}_$rep 200 $B --input logits-bf16 --vocab 256000 --tokens 4 --q1-shape $sh
    step f32_128256_s${sh}_$rep 200 $B --input logits-f32 --vocab 128256 --tokens 4 --q1-shape $sh
    step f32_151936_s${sh}_$rep 200 $B --input logits-f32 --vocab 151936 --tokens 4 --q1-shape $sh
    step f32_262144_s${sh}_$rep 200 $B --input logits-f32 --vocab 262144 --tokens 4 --q1-shape $sh
  done
done
python3 tools/sessions/ab/summ.py $o
echo "== done"
