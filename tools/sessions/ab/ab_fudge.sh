# Division-free fudged decode: parity tests, then A/B vs tools/sessions/ab/liblac_r03_fudge0.so on
# llama-scale u64 tables (fudged at prec 48), same box, two rounds.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/ab_fudge
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_flush.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_fudge/tests.log 2>&1 || { tail -30 gpurun_out/ab_fudge/tests.log; exit 3; }
tail -3 gpurun_out/ab_fudge/tests.log
for r in 1 2; do
  for v in old new; do
    lib=lac_amd/liblac.so; [ $v = old ] && lib=tools/sessions/ab/liblac_r03_fudge0.so
    LAC_LIB=$lib timeout -k 10 300 python3 bench.py --cpu-baseline off --pmf-bits 64 --steps 10 > gpurun_out/ab_fudge/u64_${v}_$r.json 2>/dev/null || exit 3
  done
done
python3 tools/sessions/ab/summ.py gpurun_out/ab_fudge
