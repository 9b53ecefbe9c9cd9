#!/bin/bash
# rocprofv3 evidence for the bench lines (run on the GPU box via gpurun):
#   kernel-trace + stats of the pmf headline and the bf16 logits bench, then one
#   FETCH_SIZE PMC pass each (separate runs: counters never share a run with tracing).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {   # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "== $name"
    timeout -s KILL "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log"
    [ $rc -ne 0 ] && exit $rc
    return 0
}
B="python3 bench.py --cpu-baseline off"
step stats_pmf 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pmf -o run --output-format csv -- $B --steps 10 --warmup 2
step stats_bf16 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bf16 -o run --output-format csv -- $B --steps 10 --warmup 2 --input logits-bf16
step pmc_pmf 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_pmf -o run --output-format csv -- $B --steps 3 --warmup 1
step pmc_bf16 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_bf16 -o run --output-format csv -- $B --steps 3 --warmup 1 --input logits-bf16
echo "== done"
