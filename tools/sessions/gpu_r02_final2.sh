#!/bin/bash
# Round-2 evidence on one MI355X (gpurun): GPU tests, smoke, the headline bench with
# its CPU baseline, rocprofv3 kernel stats + FETCH_SIZE passes (separate runs) of
# the pmf headline and the bf16 logits bench, and the secondary bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r02final2}; mkdir -p $o
step() {   # step <name> <seconds> <cmd...>: any failure ends the session
    local name=$1 secs=$2; shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "$o/$name.out" 2> "$o/$name.err"
    local rc=$?
    echo "== $name rc=$rc"; tail -n 2 "$o/$name.out" | cut -c1-300
    [ $rc -ne 0 ] && { tail -n 20 "$o/$name.err"; exit $rc; }
    return 0
}
B="python3 bench.py --cpu-baseline off"
step tests 600 python3 -u -m pytest tests -m gpu -q -x -rf --timeout 120 --timeout-method thread
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench_c3 300 python3 bench.py
step stats_pmf 300 rocprofv3 --kernel-trace --stats -d $o/prof_pmf -o run --output-format csv -- $B --steps 10 --warmup 2
step stats_bf16 300 rocprofv3 --kernel-trace --stats -d $o/prof_bf16 -o run --output-format csv -- $B --steps 10 --warmup 2 --input logits-bf16
step pmc_pmf 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $o/pmc_pmf -o run --output-format csv -- $B --steps 3 --warmup 1
step pmc_bf16 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $o/pmc_bf16 -o run --output-format csv -- $B --steps 3 --warmup 1 --input logits-bf16
step bench_u64 300 $B --pmf-bits 64 --steps 10
step bench_c4 300 $B --vocab 128256 --steps 5
step bench_bf16 300 $B --input logits-bf16
step bench_f32 300 $B --input logits-f32
step bench_bf16_c4 300 $B --input logits-bf16 --vocab 128256 --steps 5
step bench_f32_v64k 300 $B --input logits-f32 --vocab 65536 --steps 5
step bench_f32_c4 300 $B --input logits-f32 --vocab 128256 --steps 5 --tokens 8
step stats_f32c4 300 rocprofv3 --kernel-trace --stats -d $o/prof_f32c4 -o run --output-format csv -- $B --steps 5 --warmup 2 --input logits-f32 --vocab 128256 --tokens 8
step pmc_f32c4 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $o/pmc_f32c4 -o run --output-format csv -- $B --steps 3 --warmup 1 --input logits-f32 --vocab 128256 --tokens 8
echo "== done"
