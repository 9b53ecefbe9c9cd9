#!/bin/bash
# Round 4: the whole GPU suite on the uniform decode step, then the decode baselines.
#   gpurun -- bash tools/sessions/gpu_r04_c.sh [outdir]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r04c}; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log
case $rc in 0) ;; *) echo "tests rc=$rc"; exit 3;; esac
bash tools/sessions/gpu_r04_base.sh ${1:-r04c}/base
