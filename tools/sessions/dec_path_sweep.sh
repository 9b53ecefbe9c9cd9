# decode path A/B at few streams (stats vs block), same box, one process per point
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/s3
for B in ${SWEEP_B:-4 16 64 256 1024}; do
  T=$(( B >= 256 ? 32 : 64 ))
  for p in stats block; do
    timeout -k 10 200 python3 bench.py --steps ${SWEEP_STEPS:-2} --warmup 1 --cpu-baseline off --streams $B --tokens $T --decode-path $p \
      > gpurun_out/s3/B${B}_$p.json 2>/dev/null || exit 3
  done
done
echo done
