#!/bin/bash
# pmf decode at few streams (stats path, AUTO below 1536 streams outside 160-256): the lean
# step (in-tree) vs k_decode_seq alone (-DLAC_LEAN=0).  gpurun -- bash tools/sessions/ab/ab_r04_fewstreams.sh <outdir>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/${1:-fewstreams}; mkdir -p $o
for B in ${BS:-4 16 64 512 1024}; do
    for v in ${VS:-cur nolean}; do
        L=; [ $v != cur ] && L=tools/_probe/liblac_$v.so
        timeout -k 10 200 env ${L:+LAC_LIB=$L} python3 bench.py --cpu-baseline off --streams $B --tokens 512 --steps 3 --warmup 2 --decode-reps 3 > $o/b${B}_$v.json 2> $o/b${B}_$v.err || { tail -20 $o/b${B}_$v.err; exit 1; }
        python3 -c "import json; d=json.loads(open('$o/b${B}_$v.json').read().strip().splitlines()[-1]); p=d['parity']['decode']; print('B=$B $v', round(p['symbols_per_s']/1e6, 3), 'M sym/s', {k: round(1e3*x, 3) for k, x in p['kernel_ms_per_step_each'].items()}, 'rt', d['parity']['round_trip_all_streams'])"
    done
done
