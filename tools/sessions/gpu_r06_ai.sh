#!/bin/bash
# Round 6: is the bf16 decode-form row statistics' 78 % -> 84 % a matter of the box's state?
# tools/q1_b2b.py (bf16 c3, back to back) four times in a row with one library, then the
# bf16 c3 bench line twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06ai}; mkdir -p $o
for rep in 1 2 3 4; do
    timeout -k 10 300 python3 tools/q1_b2b.py --vocab 32000 --reps 20 > $o/b2b_$rep.json 2> $o/b2b.err || exit 3
    date +%s.%N >> $o/times.txt
done
for rep in 1 2; do
    timeout -k 10 300 python3 bench.py --input logits-bf16 --cpu-baseline off --decode-reps 20 > $o/bf16_$rep.json 2> $o/bf16.err || exit 3
done
for f in $o/b2b_*.json; do echo "$(basename $f) $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print([(k, round(v["q1_stats_ms_per_launch"],4), round(v["frac_of_8TBps"],3), round(v.get("q1_decode_us_per_step") or 0,2)) for k, v in d.items() if isinstance(v, dict)])' $f)"; done
for f in $o/bf16_*.json; do python3 -c "
import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']['decode']
print('$(basename $f)', 'enc %.2f' % (d['value']/1e6), 'dec %.2f M sym/s' % (p['symbols_per_s']/1e6), p.get('kernel_ms_per_step_each'))"; done
