#!/bin/bash
# Same-box A/B of the bf16 row-group encode form's register fixes: tools/sessions/ab/liblac_base.so vs lac_amd/liblac.so.
set -u
cd "${GRAFT_REPO_ROOT}"
out=gpurun_out/${1:-ab_groups_bf16}; mkdir -p $out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_logits.py -q -x --timeout 120 --timeout-method thread > $out/tests.txt 2>&1 || exit 3
for r in 1 2; do
  for v in base new; do
    lib=lac_amd/liblac.so; [ $v != new ] && lib=tools/sessions/ab/liblac_$v.so
    for cfg in "bf16_256k:--vocab 256000" "bf16_152k:--vocab 151936" "bf16_262k:--vocab 262144"; do
      name=${cfg%%:*}; args=${cfg#*:}
      LAC_LIB=$lib timeout -k 10 200 python3 bench.py --cpu-baseline off --input logits-bf16 --steps 5 --warmup 5 --tokens 8 $args > $out/${name}_${v}_$r.json 2>$out/${name}_${v}_$r.err || exit 3
    done
  done
done
echo done
