#!/bin/bash
# Round 3: device reciprocal probe, the whole GPU suite + smoke on the MI355X.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/rcp_probe > gpurun_out/rcp_probe.json 2>&1 || exit $?
cat gpurun_out/rcp_probe.json
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_all.log 2>&1
rc=$?
tail -15 gpurun_out/r03_all.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/r03_all.log 2>&1
rc=$?
tail -2 gpurun_out/r03_all.log
exit $rc
