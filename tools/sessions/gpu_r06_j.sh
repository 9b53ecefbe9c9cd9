#!/bin/bash
# Round 6: SQ counters of the two lean-step forms on bench.py's c2 workload (u32 and u64),
# from saved inputs (no torch RNG kernel in the profiled process): chunk form (commit
# c1d605c, tools/_probe/liblac_chunk.so) vs per-iteration bounds (this tree).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06j}; mkdir -p $o
B="bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 3 --warmup 1 --decode-reps 2"
timeout -k 10 200 python3 $B --save-inputs /tmp/c2in > $o/save.json 2> $o/save.err || exit 3
timeout -k 10 200 python3 $B --pmf-bits 64 --save-inputs /tmp/c2in64 > $o/save64.json 2> $o/save64.err || exit 3
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH"
S2="SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY"
n=0
for lib in lac_amd/liblac.so tools/_probe/liblac_chunk.so; do
  tag=$(basename $lib .so)
  for inp in c2in c2in64; do
    bits=32; [ $inp = c2in64 ] && bits=64
    LAC_LIB=$lib timeout -k 10 200 python3 $B --pmf-bits $bits --load-inputs /tmp/$inp > $o/${tag}_${inp}.json 2> $o/${tag}_${inp}.err || exit 3
    for set in "$S1" "$S2"; do
      n=$((n+1))
      LAC_LIB=$lib timeout -s KILL 180 rocprofv3 --pmc $set --kernel-trace -d $o/pmc_${tag}_${inp}_$n -o run --output-format csv -- python3 $B --pmf-bits $bits --load-inputs /tmp/$inp > $o/pmc_$n.json 2> $o/pmc_$n.err
      rc=$?; echo "pmc $tag $inp pass $n rc=$rc"; [ $rc -eq 0 ] || exit 3
    done
    python3 tools/pmc_summary.py $o k_decode_lean > /dev/null
  done
done
for f in $o/liblac_*.json; do python3 -c "
import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']
print('$f', 'dec us/step %.3f' % (1e3*p['decode']['kernel_ms_per_step']), 'exact', p.get('bit_exact_vs_oracle'), 'rt', p.get('round_trip_all_streams'))"; done
for d in $o/pmc_*; do [ -d $d ] && echo "== $d" && python3 tools/pmc_summary.py $d k_decode_lean; done
