#!/bin/bash
# Round 3: the one-row-per-CU register shape (22) -- parity tests, then same-box A/B
# against AUTO (row groups) at bf16 Qwen2 / 131080 and f32 65540.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-wide}; mkdir -p $o
step() {   # step <name> <seconds> <cmd...>: any failure ends the session
    local name=$1 secs=$2; shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "$o/$name.out" 2> "$o/$name.err"
    local rc=$?
    echo "== $name rc=$rc"; tail -n 3 "$o/$name.out" | cut -c1-400
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
# u64 fine decode with fewer VALU ops per element (saturating high-word sum, min3 keys)
for rep in 1 2; do
  for v in head new; do
    lib=lac_amd/liblac.so; [ $v = head ] && lib=tools/sessions/ab/liblac_r03_head.so
    step u64_${v}_$rep 300 env LAC_LIB=$lib $B --pmf-bits 64
    step u64s31_${v}_$rep 300 env LAC_LIB=$lib $B --pmf-bits 64 --scale-bits 31
  done
done
step all_tests 900 python3 -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
echo "== done"
