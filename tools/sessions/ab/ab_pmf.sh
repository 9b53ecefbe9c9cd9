# Same-box A/B of tools/sessions/ab/liblac_base.so against lac_amd/liblac.so on the pmf path
# (c3 u32 headline, c3 u64, c4 u32): encode + decode.
set -u
cd "${GRAFT_REPO_ROOT}"
out=gpurun_out/ab_pmf; mkdir -p $out
for r in 1 2; do
  for v in base new; do
    lib=lac_amd/liblac.so; [ $v = base ] && lib=tools/sessions/ab/liblac_base.so
    for cfg in "c3:" "u64:--pmf-bits 64 --steps 10" "c4:--vocab 128256 --steps 5"; do
      name=${cfg%%:*}; args=${cfg#*:}
      LAC_LIB=$lib timeout -k 10 200 python3 bench.py --cpu-baseline off $args > $out/${name}_${v}_$r.json 2>$out/${name}_${v}_$r.err || exit 3
    done
  done
done
echo done
