# u64 decode: llama-scale (fudged at prec 48) vs 2^31-scale (unfudged) tables in u64 storage
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/u64probe
for k in 60 31 40; do
  timeout -k 10 300 python3 bench.py --cpu-baseline off --pmf-bits 64 --scale-bits $k --steps 10 > gpurun_out/u64probe/u64_s$k.json 2>/dev/null || exit 3
done
python3 tools/sessions/ab/summ.py gpurun_out/u64probe
