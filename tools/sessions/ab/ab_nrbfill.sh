#!/bin/bash
# The register + LDS-slot forms at the same fill (93.75 % of their capacity), bf16, no groups:
# 4 rows per block (17), 2 rows (18), 1 row (15).
set -u
cd "${GRAFT_REPO_ROOT}"
out=gpurun_out/ab_nrbfill; mkdir -p $out
for r in 1 2; do
  for cfg in "s17:--vocab 30720 --q1-shape 17" "s18:--vocab 61440 --q1-shape 18" "s15:--vocab 122880 --q1-shape 15" \
             "s15full:--vocab 128256 --q1-shape 15"; do
    name=${cfg%%:*}; args=${cfg#*:}
    timeout -k 10 200 python3 bench.py --cpu-baseline off --steps 5 --warmup 5 --tokens 8 --decode-reps 1 --input logits-bf16 $args > $out/${name}_$r.json 2>$out/${name}_$r.err || exit 3
  done
done
python3 tools/sessions/ab/summ.py $out
