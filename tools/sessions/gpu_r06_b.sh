#!/bin/bash
# Round 6: the new tests of the round's first commit (set_output refusal, one-generator
# tables, untraced straight-form goldens) and the --gather bench line (per-job symbol
# variants, every held job checked).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06b}; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_dist.py tests/test_gpu_api.py::test_synth_tables_one_generator_equal_per_step_generators \
    tests/test_gpu_parity.py -k "set_output or synth or untraced or golden or kat1" > $o/tests.log 2>&1
rc=$?; tail -5 $o/tests.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python3 bench.py --gather --cpu-baseline off > $o/gather_w1.json 2> $o/gather_w1.err || exit 3
python3 -c "
import json; d=json.loads([l for l in open('$o/gather_w1.json') if l.startswith('{')][-1]); p=d['parity']
print('gather', d['value']/1e6, p.get('gather_ok'), p['gather'], p['bit_exact_vs_oracle'])"
