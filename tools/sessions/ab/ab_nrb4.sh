#!/bin/bash
# Where the 4-row group form loses: bf16 rows of the same shape without groups (shape 17
# forced at 3840 / 4032 / 4096 vectors) and Qwen2 without the exchange wait (nowait2).
set -u
cd "${GRAFT_REPO_ROOT}"
out=gpurun_out/ab_nrb4; mkdir -p $out
for r in 1 2; do
  for cfg in "new:q152k:--vocab 151936" "nowait2:q152k:--vocab 151936" "new:s17_3840:--vocab 30720 --q1-shape 17" \
             "new:s17_4032:--vocab 32256 --q1-shape 17" "new:s17_4096:--vocab 32768 --q1-shape 17" \
             "new:auto_4032:--vocab 32256"; do
    v=${cfg%%:*}; rest=${cfg#*:}; name=${rest%%:*}; args=${rest#*:}
    lib=lac_amd/liblac.so; [ $v != new ] && lib=tools/sessions/ab/liblac_$v.so
    LAC_LIB=$lib timeout -k 10 200 python3 bench.py --cpu-baseline off --steps 5 --warmup 5 --tokens 8 --decode-reps 1 --input logits-bf16 $args > $out/${name}_${v}_$r.json 2>$out/${name}_${v}_$r.err || exit 3
  done
done
python3 tools/sessions/ab/summ.py $out
