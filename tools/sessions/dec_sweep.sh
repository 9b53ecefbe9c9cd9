#!/bin/bash
# Decode-path sweep on the GPU box: tools/sessions/dec_sweep.sh "<streams> <tokens> <path>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/dec
for spec in "$@"; do
    set -- $spec
    B=$1; T=$2; P=$3; shift 3
    tag=$(echo "$*" | tr -c 'A-Za-z0-9' '_')
    out=gpurun_out/dec/B${B}_T${T}_${P}${tag:+_$tag}.json
    timeout -k 10 180 python3 bench.py --streams "$B" --tokens "$T" --decode-path "$P" --steps 3 --warmup 1 \
        --cpu-baseline off "$@" > "$out" 2> "${out%.json}.err"
    rc=$?
    [ $rc -ne 0 ] && { echo "$spec rc=$rc"; tail -5 "${out%.json}.err"; exit $rc; }
    python3 -c "import json; d=json.load(open('$out')); p=d['parity']; q=p['decode']; print('B=$B T=$T $P', 'enc', round(d['value']/1e6,3), 'Msym/s  dec', round(q['symbols_per_s']/1e6,3), 'Msym/s', q['kernel'], round(q['kernel_ms_per_step']*1e3,1), 'us/step', p['round_trip_all_streams'], p['bit_exact_vs_oracle'])"
done
