#!/bin/bash
# Same-box A/B of the deferred DEC chunk-total store (LAC_Q1_DEFER): q1 row-stats
# device time per direction, alternating encode / decode (tools/q1_encdec_alt.py).
set -u
cd "${GRAFT_REPO_ROOT}"
out=gpurun_out/${1:-ab_defer}; mkdir -p $out
for r in 1 2; do
  for v in nodefer new; do
    lib=lac_amd/liblac.so; [ $v != new ] && lib=tools/sessions/ab/liblac_$v.so
    for cfg in "bf16c4:--input logits-bf16 --vocab 128256" "f32c4:--input logits-f32 --vocab 128256 --tokens 8" \
               "bf16c3:--input logits-bf16 --vocab 32000" "f32c3:--input logits-f32 --vocab 32000"; do
      name=${cfg%%:*}; args=${cfg#*:}
      LAC_LIB=$lib timeout -k 10 200 python3 tools/q1_encdec_alt.py --reps 3 $args > $out/${name}_${v}_$r.jsonl 2>$out/${name}_${v}_$r.err || exit 3
    done
  done
done
echo done
