#!/bin/bash
# Timing experiment: row groups without the maximum exchange (wrong tables) vs the real thing.
set -u
cd "${GRAFT_REPO_ROOT}"
out=gpurun_out/ab_nowait; mkdir -p $out
for r in 1 2; do
  for v in nowait new; do
    lib=lac_amd/liblac.so; [ $v != new ] && lib=tools/sessions/ab/liblac_$v.so
    for cfg in "bf16_152k:--input logits-bf16 --vocab 151936" "bf16_131k:--input logits-bf16 --vocab 131080" \
               "bf16_262k:--input logits-bf16 --vocab 262144" "f32_65540:--input logits-f32 --vocab 65540" \
               "f32_128k:--input logits-f32 --vocab 128256"; do
      name=${cfg%%:*}; args=${cfg#*:}
      LAC_LIB=$lib timeout -k 10 200 python3 bench.py --cpu-baseline off --steps 5 --warmup 5 --tokens 8 --decode-reps 1 $args > $out/${name}_${v}_$r.json 2>$out/${name}_${v}_$r.err || exit 3
    done
  done
done
python3 tools/sessions/ab/summ.py $out
