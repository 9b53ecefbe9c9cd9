#!/bin/bash
# Round 3 final check on the committed library: whole GPU suite + smoke, the headline
# bench with its CPU baseline, rocprofv3 stats + FETCH_SIZE of the headline, and the
# logits lines the round changed.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-final}; mkdir -p $o
step() {   # step <name> <seconds> <cmd...>: any failure ends the session
    local name=$1 secs=$2; shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "$o/$name.json" 2> "$o/$name.err"
    local rc=$?
    echo "== $name rc=$rc"; tail -n 2 "$o/$name.json" | cut -c1-240
    [ $rc -ne 0 ] && { tail -n 30 "$o/$name.err"; exit $rc; }
    return 0
}
step tests 900 python3 -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench_c3 300 python3 bench.py
step stats_pmf 300 rocprofv3 --kernel-trace --stats -d $o/prof_pmf -o run --output-format csv -- python3 bench.py --cpu-baseline off --steps 10 --warmup 2
step pmc_pmf 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $o/pmc_pmf -o run --output-format csv -- python3 bench.py --cpu-baseline off --steps 3 --warmup 1
B="python3 bench.py --cpu-baseline off --steps 10 --warmup 5"
step bf16_c3 200 $B --input logits-bf16
step bf16_qwen2 200 $B --input logits-bf16 --vocab 151936 --tokens 8
step bf16_llama4 200 $B --input logits-bf16 --vocab 202048 --tokens 4
step f32_deepseek 200 $B --input logits-f32 --vocab 102400 --tokens 4
step u64 200 $B --pmf-bits 64
step c2 200 $B --streams 1 --tokens 4096 --steps 5 --warmup 2
echo "== done"
