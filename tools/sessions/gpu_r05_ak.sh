#!/bin/bash
# Round 5: the first default bench on a fresh box reads ~2.5 % below later ones
# (52.4 vs 53.8 M sym/s): four headline runs in a row, one with 100 warm jobs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05ak}; mkdir -p $o
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 3
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --cpu-baseline off > $o/def$r.json 2> $o/def$r.err || exit 3
done
timeout -k 10 300 python3 bench.py --cpu-baseline off --warmup 100 > $o/w100.json 2> $o/w100.err || exit 3
timeout -k 10 300 python3 bench.py --cpu-baseline off > $o/def3.json 2> $o/def3.err || exit 3
for f in def1 def2 w100 def3; do python3 -c "
import json; d=json.loads([l for l in open('$o/$f.json') if l.startswith('{')][-1]); r=d['roofline']
print('$f', '%.3f M sym/s' % (d['value']/1e6), 'ms/step %.4f' % d['ms_per_step'], 'kernel %.4f' % r['kernel_ms_per_launch'], 'frac', round(r['frac'],4))"; done
