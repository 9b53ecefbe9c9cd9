#!/bin/bash
# SQ / TCC counters of any python3 command, one rocprofv3 --pmc pass per counter set
# (kernel trace only, never combined with other tracing):
#   tools/sessions/pmc_passes.sh <outdir> <python3 script and args...>
# then: python3 tools/pmc_summary.py gpurun_out/<outdir>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/$1; shift
mkdir -p "$out"
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES" \
           "SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM" \
           "FETCH_SIZE"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $set --kernel-trace -d "$out/p$i" -o run --output-format csv -- \
        python3 "$@" > "$out/p$i.log" 2>&1
    rc=$?
    echo "pass $i rc=$rc"
    [ $rc -ne 0 ] && { tail -20 "$out/p$i.log"; exit $rc; }
done
exit 0
