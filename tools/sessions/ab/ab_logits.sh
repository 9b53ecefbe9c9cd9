# Same-box A/B of tools/sessions/ab/liblac_base.so (the library before a change) against
# lac_amd/liblac.so on the logits path: c3 / c4 shapes, bf16 / f32, encode + decode.
#   tools/sessions/ab/liblac_base.so: hipcc ... lac_amd/csrc/lac_kernels.hip -o tools/sessions/ab/liblac_base.so at the base commit
set -u
cd "${GRAFT_REPO_ROOT}"
out=gpurun_out/ab_logits; mkdir -p $out
for r in 1 2; do
  for v in base new; do
    lib=lac_amd/liblac.so; [ $v = base ] && lib=tools/sessions/ab/liblac_base.so
    for cfg in "bf16c3:--input logits-bf16" "f32c3:--input logits-f32" \
               "bf16c4:--input logits-bf16 --vocab 128256 --steps 5" "f32c4:--input logits-f32 --vocab 128256 --steps 5 --tokens 8"; do
      name=${cfg%%:*}; args=${cfg#*:}
      LAC_LIB=$lib timeout -k 10 200 python3 bench.py --cpu-baseline off $args > $out/${name}_${v}_$r.json 2>$out/${name}_${v}_$r.err || exit 3
    done
  done
done
echo done
