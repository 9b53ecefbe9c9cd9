set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/slots
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_logits.py -x -v --timeout 300 --timeout-method thread > gpurun_out/slots/logits_tests.log 2>&1 || { tail -30 gpurun_out/slots/logits_tests.log; exit 3; }
tail -3 gpurun_out/slots/logits_tests.log
OUT=ab_rbo VARIANTS="base norb new" bash tools/sessions/ab/ab_slots.sh
