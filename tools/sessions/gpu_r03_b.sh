#!/bin/bash
# Round 3: contention test for row groups, c2 test, fudge A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r03b
timeout -k 10 60 ./tools/rcp_probe > gpurun_out/r03b/rcp_probe_after.json 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest tests/test_gpu_logits.py -k "cus or paired" tests/test_gpu_parity.py::test_c2_shape_one_stream_4096_steps -x -v --timeout 300 --timeout-method thread > gpurun_out/r03b/tests.log 2>&1 || { tail -40 gpurun_out/r03b/tests.log; exit 3; }
tail -12 gpurun_out/r03b/tests.log
bash tools/sessions/ab/ab_fudge.sh
