#!/bin/bash
# Round 6 (after the lean step's second pass): SQ counters of the lean step alone (a build without the L2-prefetching helper waves, so the
# counts are the decoder wave's) on bench.py's c2 u32 / u64 workloads from saved inputs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06x}; mkdir -p $o
B="bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 3 --warmup 1 --decode-reps 2"
timeout -k 10 200 python3 $B --save-inputs /tmp/c2in > $o/save.json 2> $o/save.err || exit 3
timeout -k 10 200 python3 $B --pmf-bits 64 --save-inputs /tmp/c2in64 > $o/save64.json 2> $o/save64.err || exit 3
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH"
S2="SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY"
n=0
for inp in c2in c2in64; do
  bits=32; [ $inp = c2in64 ] && bits=64
  LAC_LIB=tools/_probe/liblac_nohelp7.so timeout -k 10 200 python3 $B --pmf-bits $bits --load-inputs /tmp/$inp > $o/nohelp_${inp}.json 2> $o/nohelp_${inp}.err || exit 3
  for set in "$S1" "$S2"; do
    n=$((n+1))
    LAC_LIB=tools/_probe/liblac_nohelp7.so timeout -s KILL 180 rocprofv3 --pmc $set --kernel-trace -d /tmp/pmc_${inp}_$n -o run --output-format csv -- python3 $B --pmf-bits $bits --load-inputs /tmp/$inp > $o/pmc_$n.json 2> $o/pmc_$n.err
    rc=$?; echo "pmc $inp pass $n rc=$rc"; [ $rc -eq 0 ] || exit 3
    python3 tools/pmc_summary.py /tmp/pmc_${inp}_$n k_decode_lean > $o/pmc_${inp}_$n.txt
    cat $o/pmc_${inp}_$n.txt
  done
done
for f in $o/nohelp_*.json; do python3 -c "
import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']
print('$f', 'dec us/step %.3f' % (1e3*p['decode']['kernel_ms_per_step']), 'exact', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'))"; done
