#!/bin/bash
# SQ counters for the logits-path kernels (separate --pmc passes, kernel trace only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/q1pmc
ARGS="${ARGS:---input logits-bf16}"
timeout -k 10 120 rocprofv3 -L > gpurun_out/q1pmc/counters.txt 2>&1 || true
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD" \
           "FETCH_SIZE"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/q1pmc/p$i -o run --output-format csv -- \
        python3 bench.py --steps 3 --warmup 1 --cpu-baseline off $ARGS > gpurun_out/q1pmc/p$i.log 2>&1
    rc=$?
    echo "pass $i rc=$rc"
    [ $rc -ne 0 ] && { tail -20 gpurun_out/q1pmc/p$i.log; exit $rc; }
done
exit 0
