# A/B only (tests already run): division-free fudged decode vs tools/sessions/ab/liblac_r03_fudge0.so, u64 llama-scale.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/ab_fudge
rm -f gpurun_out/ab_fudge/*.json
for r in 1 2; do
  for v in old new; do
    lib=lac_amd/liblac.so; [ $v = old ] && lib=tools/sessions/ab/liblac_r03_fudge0.so
    LAC_LIB=$lib timeout -k 10 300 python3 bench.py --cpu-baseline off --pmf-bits 64 --steps 10 > gpurun_out/ab_fudge/u64_${v}_$r.json 2>gpurun_out/ab_fudge/err_${v}_$r.txt || exit 3
  done
done
python3 tools/sessions/ab/summ.py gpurun_out/ab_fudge
