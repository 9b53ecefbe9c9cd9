# A/B of the reciprocal's Newton step: tools/sessions/ab/liblac_r03_rcp0.so (v_rcp_f64 alone)
# vs lac_amd/liblac.so, u64 (llama-scale) and u32 c3 decode + encode, same box, two rounds.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/ab_rcp
timeout -k 10 60 ./tools/rcp_probe > gpurun_out/ab_rcp/rcp_probe_after.txt 2>&1 || exit 3
for r in 1 2; do
  for v in old new; do
    lib=lac_amd/liblac.so; [ $v = old ] && lib=tools/sessions/ab/liblac_r03_rcp0.so
    LAC_LIB=$lib timeout -k 10 300 python3 bench.py --cpu-baseline off --pmf-bits 64 --steps 10 > gpurun_out/ab_rcp/u64_${v}_$r.json 2>/dev/null || exit 3
    LAC_LIB=$lib timeout -k 10 300 python3 bench.py --cpu-baseline off --steps 10 > gpurun_out/ab_rcp/c3_${v}_$r.json 2>/dev/null || exit 3
  done
done
python3 tools/sessions/ab/summ.py gpurun_out/ab_rcp
