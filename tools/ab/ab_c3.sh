# A/B of the round's start library vs the current one: c3 pmf and bf16 logits, encode + decode, same box
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/ab
for r in 1 2; do
  for v in old new; do
    lib=lac_amd/liblac.so; [ $v = old ] && lib=tools/ab/liblac_old.so
    LAC_LIB=$lib timeout -k 10 300 python3 bench.py --cpu-baseline off --steps 10 > gpurun_out/ab/c3_${v}_$r.json 2>/dev/null || exit 3
    LAC_LIB=$lib timeout -k 10 300 python3 bench.py --cpu-baseline off --steps 10 --input logits-bf16 > gpurun_out/ab/bf16_${v}_$r.json 2>/dev/null || exit 4
  done
done
echo done
