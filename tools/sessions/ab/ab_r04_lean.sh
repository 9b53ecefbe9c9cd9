#!/bin/bash
# c2 decode A/B: k_decode_lean (in-tree liblac) vs k_decode_seq alone (LAC_LEAN=0 build),
# then the decode-path GPU tests on the lean build.  gpurun -- bash tools/sessions/ab/ab_r04_lean.sh [outdir]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-ab_lean}; mkdir -p $o
step() {
    local name=$1 secs=$2; shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "$o/$name.json" 2> "$o/$name.err"
    local rc=$?
    echo "== $name rc=$rc"
    python3 -c "import json,sys
try:
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p = d.get('parity', {}).get('decode', {})
    print(sys.argv[2], 'value', round(d['value']), 'dec_us_per_step', round(1e3 * p.get('kernel_ms_per_step', 0), 3), 'each', [round(x) for x in p.get('symbols_per_s_each', [])], 'rt', d.get('parity', {}).get('round_trip_all_streams'))
except Exception as e:
    print(sys.argv[2], open(sys.argv[1]).read()[-300:])" "$o/$name.json" $name
    [ $rc -ne 0 ] && { tail -n 30 "$o/$name.err"; exit $rc; }
    return 0
}
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 5 --warmup 2 --decode-reps 5"
step tests_dec 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_checkpoint.py -m gpu -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider
for r in 1 2; do
    step c2_lean_$r 200 $C2
    step c2_seq_$r 200 env LAC_LIB=tools/_probe/liblac_nolean.so $C2
    step c2_nolim_$r 200 env LAC_LIB=tools/_probe/liblac_lean_nolim.so $C2
    step c2_8mb_$r 200 env LAC_LIB=tools/_probe/liblac_lean_8mb.so $C2
done
B64="python3 bench.py --cpu-baseline off --streams 64 --tokens 256 --steps 5 --warmup 2 --decode-reps 5"
step b64_lean 200 $B64
step b64_seq 200 env LAC_LIB=tools/_probe/liblac_nolean.so $B64
step prof_c2 200 rocprofv3 --kernel-trace --stats -d $o/prof_c2 -o run --output-format csv -- python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 3 --warmup 1 --decode-reps 2
find $o/prof_c2 -type f ! -name '*stats.csv' -delete
echo "== done"
