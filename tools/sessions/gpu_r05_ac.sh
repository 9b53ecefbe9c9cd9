#!/bin/bash
# Round 5: SQ counters of the c2 lean decode step alone (helpers off:
# tools/_probe/liblac_nohelp.so, so the kernel's waves are the decoder's), 2 passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05ac}; mkdir -p $o
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC"; do
    i=$((i+1))
    LAC_LIB=tools/_probe/liblac_nohelp.so timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d $o/d$i -o run --output-format csv -- python3 tools/dec_phase_probe.py --one-generator > $o/d$i.log 2>&1
    rc=$?
    echo "pass $i rc=$rc"
    [ $rc -ne 0 ] && { grep -v "^    @" $o/d$i.log | tail -5; exit 3; }
done
exit 0
