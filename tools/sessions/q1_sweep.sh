#!/bin/bash
# Logits-path shape sweep on the GPU box: tools/sessions/q1_sweep.sh "<input> <shape>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/q1
for spec in "$@"; do
    set -- $spec
    inp=$1; shp=$2; shift 2
    out=gpurun_out/q1/sweep_${inp}_${shp}.json
    timeout -k 10 120 python3 bench.py --input "$inp" --q1-shape "$shp" --steps 10 --warmup 2 --cpu-baseline off "$@" \
        > "$out" 2> "${out%.json}.err"
    rc=$?
    [ $rc -ne 0 ] && { echo "$inp $shp rc=$rc"; tail -5 "${out%.json}.err"; exit $rc; }
    python3 -c "import json; d=json.load(open('$out')); r=d['roofline']; p=d['parity']; print('$inp shape=$shp', round(d['value']/1e6,2), 'Msym/s stats', round(r['kernel_ms_per_launch'],4), 'ms', round(r['frac'],3), 'steps', {k: round(v,4) for k,v in r['kernel_ms_per_step'].items()}, 'dec', round(p['decode']['symbols_per_s']/1e6,2), 'Msym/s', p['bit_exact_vs_oracle'], p['round_trip_all_streams'])"
done
