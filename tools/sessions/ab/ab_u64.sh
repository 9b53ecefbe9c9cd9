# A/B of the round's start library vs the current one on the u64 (fudged) and u32 decode, same box
# tools/sessions/ab/liblac_old.so: the round-start library, built by
#   git --work-tree=/tmp/old checkout 9369c7c -- lac_amd/csrc include && git reset -q HEAD -- lac_amd/csrc include
#   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I /tmp/old/include -I /tmp/old/lac_amd/csrc \
#         /tmp/old/lac_amd/csrc/lac_kernels.hip -o tools/sessions/ab/liblac_old.so
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/ab
for r in 1 2; do
  for v in old new; do
    lib=lac_amd/liblac.so; [ $v = old ] && lib=tools/sessions/ab/liblac_old.so
    LAC_LIB=$lib timeout -k 10 300 python3 bench.py --cpu-baseline off --pmf-bits 64 --steps 5 > gpurun_out/ab/u64_${v}_$r.json 2>/dev/null || exit 3
  done
done
echo done
