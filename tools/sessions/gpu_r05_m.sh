#!/bin/bash
# Round 5: few-stream encode step on the scalar unit (ult_s compares, plane_append_s,
# fewer readlanes): parity tests, c2 phase probe + plain, c2 bench, 64/256 streams.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05m}; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_checkpoint.py tests/test_gpu_logits.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/t.log 2>&1
rc=$?; tail -3 $o/t.log; [ $rc -eq 0 ] || exit 3
LAC_LIB=tools/_probe/liblac_encphases.so timeout -k 10 200 python3 tools/enc_phase_probe.py > $o/enc_phases.json 2> $o/enc_phases.err || exit 3
cat $o/enc_phases.json
timeout -k 10 200 python3 tools/enc_phase_probe.py > $o/enc_plain.json 2> $o/enc_plain.err || exit 3
cat $o/enc_plain.json
LAC_LIB=tools/_probe/liblac_presplit.so timeout -k 10 200 python3 tools/enc_phase_probe.py > $o/enc_base.json 2> $o/enc_base.err || exit 3
cat $o/enc_base.json
timeout -k 10 300 python3 bench.py --streams 1 --tokens 4096 --steps 3 --warmup 1 --cpu-baseline off > $o/c2.json 2> $o/c2.err || exit 3
for Bn in 64 256; do
  timeout -k 10 300 python3 bench.py --streams $Bn --tokens 256 --steps 3 --warmup 1 --cpu-baseline off > $o/b$Bn.json 2> $o/b$Bn.err || exit 3
  LAC_LIB=tools/_probe/liblac_presplit.so timeout -k 10 300 python3 bench.py --streams $Bn --tokens 256 --steps 3 --warmup 1 --cpu-baseline off > $o/b${Bn}_base.json 2> $o/b${Bn}_base.err || exit 3
done
for f in c2 b64 b64_base b256 b256_base; do python3 -c "
import json
j=json.loads([l for l in open('$o/$f.json') if l.startswith('{')][-1])
print('$f', round(j['value']/1e6,3), 'M sym/s', j['roofline']['kernel_ms_per_step'], 'dec', round(j['parity']['decode']['symbols_per_s']/1e6,3), j['parity']['round_trip_all_streams'], j['parity']['bit_exact_vs_oracle'])
"; done
# few-stream decode: the sign tests through SCC (probe build) vs the product build
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --streams 1 --tokens 4096 --steps 2 --warmup 1 --cpu-baseline off --decode-reps 3 > $o/c2dec_prod$r.json 2> $o/c2dec_prod$r.err || exit 3
  LAC_LIB=tools/_probe/liblac_decscc.so timeout -k 10 300 python3 bench.py --streams 1 --tokens 4096 --steps 2 --warmup 1 --cpu-baseline off --decode-reps 3 > $o/c2dec_scc$r.json 2> $o/c2dec_scc$r.err || exit 3
done
for f in c2dec_prod1 c2dec_scc1 c2dec_prod2 c2dec_scc2; do python3 -c "
import json
j=json.loads([l for l in open('$o/$f.json') if l.startswith('{')][-1])
d=j['parity']['decode']
print('$f', 'dec us/step', round(1e6/d['symbols_per_s'],3), d['kernel_ms_per_step_each'], j['parity']['round_trip_all_streams'])
"; done
