# A/B of the round's start library vs the current one on the u64 (fudged) and u32 decode, same box
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/ab
for r in 1 2; do
  for v in old new; do
    lib=lac_amd/liblac.so; [ $v = old ] && lib=tools/ab/liblac_old.so
    LAC_LIB=$lib timeout -k 10 300 python3 bench.py --cpu-baseline off --pmf-bits 64 --steps 5 > gpurun_out/ab/u64_${v}_$r.json 2>/dev/null || exit 3
  done
done
echo done
