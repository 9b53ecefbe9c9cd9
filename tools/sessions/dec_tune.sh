#!/bin/bash
# Decode-kernel variants (tools/tune/liblac_<v>.so built by tune_encode.sh build) on
# the bench workload: one dec_bench line per variant and configuration.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/dtune
for so in tools/tune/liblac_*.so; do
  v=$(basename "$so" .so)
  for cfg in "--pmf-bits 32" "--pmf-bits 64" ${DEC_EXTRA_CFG:-}; do
    tag=$(echo "$cfg" | tr -d ' -')
    LAC_LIB="$PWD/$so" timeout -k 10 200 python3 tools/dec_bench.py $cfg --reps 3 \
        > "gpurun_out/dtune/$v.$tag.json" 2> "gpurun_out/dtune/$v.$tag.err"
    rc=$?
    [ $rc -ne 0 ] && { echo "$v $cfg rc=$rc"; tail -5 "gpurun_out/dtune/$v.$tag.err"; exit $rc; }
    echo "$v $cfg $(cat gpurun_out/dtune/$v.$tag.json)"
  done
done
