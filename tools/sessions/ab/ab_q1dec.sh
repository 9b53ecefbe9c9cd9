#!/bin/bash
# Same-box A/B of k_q1_decode changes: tools/sessions/ab/liblac_base.so vs lac_amd/liblac.so,
# alternating encode / decode (tools/q1_encdec_alt.py), bf16 / f32 at c3 and c4.
set -u
cd "${GRAFT_REPO_ROOT}"
out=gpurun_out/${1:-ab_q1dec}; mkdir -p $out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_logits.py -q -x --timeout 120 --timeout-method thread > $out/tests.txt 2>&1 || exit 3
for r in 1 2; do
  for v in base new; do
    lib=lac_amd/liblac.so; [ $v != new ] && lib=tools/sessions/ab/liblac_$v.so
    for cfg in "bf16c3:--input logits-bf16 --vocab 32000" "bf16c4:--input logits-bf16 --vocab 128256" \
               "f32c4:--input logits-f32 --vocab 128256 --tokens 8"; do
      name=${cfg%%:*}; args=${cfg#*:}
      LAC_LIB=$lib timeout -k 10 200 python3 tools/q1_encdec_alt.py --reps 3 $args > $out/${name}_${v}_$r.jsonl 2>$out/${name}_${v}_$r.err || exit 3
    done
  done
done
echo done
