#!/bin/bash
# Same-box A/B of the fine decoder's occupancy bound (LAC_DECF_MINW 2 / 3 / 4) at c3 u32 and u64.
set -u
cd "${GRAFT_REPO_ROOT}"
out=gpurun_out/${1:-ab_decf}; mkdir -p $out
for r in 1 2; do
  for v in new decf3 decf4; do
    lib=lac_amd/liblac.so; [ $v != new ] && lib=tools/sessions/ab/liblac_$v.so
    for cfg in "c3:" "u64:--pmf-bits 64 --steps 10"; do
      name=${cfg%%:*}; args=${cfg#*:}
      LAC_LIB=$lib timeout -k 10 200 python3 bench.py --cpu-baseline off --warmup 5 $args > $out/${name}_${v}_$r.json 2>$out/${name}_${v}_$r.err || exit 3
    done
  done
done
echo done
