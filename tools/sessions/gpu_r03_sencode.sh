#!/bin/bash
# Round 3: the split path's serial coder chain on the scalar unit (k_encode) --
# parity tests, then same-box A/B vs the previous library at few streams (c2: one
# stream x 4096 symbols; 64 streams) and where k_encode follows the logits row stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-sencode}; mkdir -p $o
step() {   # step <name> <seconds> <cmd...>: any failure ends the session
    local name=$1 secs=$2; shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "$o/$name.json" 2> "$o/$name.err"
    local rc=$?
    echo "== $name rc=$rc"; tail -n 2 "$o/$name.json" | cut -c1-200
    [ $rc -ne 0 ] && { tail -n 30 "$o/$name.err"; exit $rc; }
    return 0
}
step tests 900 python3 -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread
B="python3 bench.py --cpu-baseline off"
for rep in 1 2; do
  for v in head new; do
    lib=lac_amd/liblac.so; [ $v = head ] && lib=tools/sessions/ab/liblac_r03_head.so
    step c2_${v}_$rep 300 env LAC_LIB=$lib $B --streams 1 --tokens 4096 --steps 5 --warmup 2
    step b64_${v}_$rep 300 env LAC_LIB=$lib $B --streams 64 --tokens 256 --steps 5 --warmup 2
    step b1024_${v}_$rep 300 env LAC_LIB=$lib $B --streams 1024 --tokens 64 --steps 5 --warmup 2
    step bf16c3_${v}_$rep 300 env LAC_LIB=$lib $B --input logits-bf16 --steps 10 --warmup 5
  done
done
python3 tools/sessions/ab/summ.py $o
echo "== done"
