#!/bin/bash
# Retired q1 shapes: the logits + fuzz GPU tests on the in-tree library, then the
# bf16 / f32 logits bench lines (AUTO unchanged, so the figures should match final6).
# gpurun -- bash tools/sessions/gpu_r04_shapes.sh <outdir>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/${1:-r04shapes}; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_logits.py tests/test_gpu_fuzz.py -m gpu -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
B="python3 bench.py --cpu-baseline off --steps 10 --warmup 5 --decode-reps 5"
run() {
    local tag=$1; shift
    timeout -k 10 200 "$@" > $o/$tag.json 2> $o/$tag.err || { tail -20 $o/$tag.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$o/$tag.json').read().strip().splitlines()[-1]); p=d['parity']['decode']; print('$tag', round(d['value']/1e6, 2), round(d['roofline']['frac'], 4), {k: round(1e3*x, 3) for k, x in p['kernel_ms_per_step_each'].items()}, 'rt', d['parity']['round_trip_all_streams'])"
}
run bf16_c3 $B --input logits-bf16
run f32_c3 $B --input logits-f32
run bf16_c4 $B --input logits-bf16 --vocab 128256
run bf16_qwen2 $B --input logits-bf16 --vocab 151936
echo "== done"
