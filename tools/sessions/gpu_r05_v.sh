#!/bin/bash
# Round 5: SQ counters of the few-stream chains (c2: one stream x 4096 steps), encode
# (k_encode) and decode, for per-step instruction counts; separate --pmc passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05v}; mkdir -p $o
C2="python3 tools/enc_phase_probe.py --one-generator"   # (4096 per-step torch generators crash under --pmc)
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_WAVES SQ_INST_CYCLES_SALU SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d $o/p$i -o run --output-format csv -- $C2 > $o/p$i.log 2>&1
    rc=$?
    echo "pass $i rc=$rc"
    [ $rc -ne 0 ] && { tail -5 $o/p$i.log; exit 3; }
done
exit 0
