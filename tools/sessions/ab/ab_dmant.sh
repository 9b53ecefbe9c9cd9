#!/bin/bash
# LDS-DMA loads of the register + slot row-stats shapes with the nt policy (new) vs without (dmant0).
set -u
cd "${GRAFT_REPO_ROOT}"
out=gpurun_out/ab_dmant; mkdir -p $out
for r in 1 2; do
  for v in dmant0 new; do
    lib=lac_amd/liblac.so; [ $v != new ] && lib=tools/sessions/ab/liblac_$v.so
    for cfg in "bf16_c4:--input logits-bf16 --vocab 128256" "f32_c4:--input logits-f32 --vocab 128256" \
               "bf16_152k:--input logits-bf16 --vocab 151936" "f32_c3:--input logits-f32 --vocab 32000" \
               "bf16_64k:--input logits-bf16 --vocab 65536" "f32_65540:--input logits-f32 --vocab 65540"; do
      name=${cfg%%:*}; args=${cfg#*:}
      LAC_LIB=$lib timeout -k 10 200 python3 bench.py --cpu-baseline off --steps 5 --warmup 5 --tokens 8 --decode-reps 1 $args > $out/${name}_${v}_$r.json 2>$out/${name}_${v}_$r.err || exit 3
    done
  done
done
python3 tools/sessions/ab/summ.py $out
