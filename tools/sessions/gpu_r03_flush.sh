#!/bin/bash
# Round 3: decoder flush / tail tests + the reference-shaped API tests on the MI355X.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_flush.py tests/test_gpu_api.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_flush.log 2>&1
rc=$?
tail -30 gpurun_out/r03_flush.log
exit $rc
