#!/bin/bash
# Round 5: k_encode with the 64-step prefetch waited for before the step loop
# (LAC_ENC_PREWAIT, product) vs the previous commit (tools/_probe/liblac_base.so): c2 and
# 64 / 256 streams interleaved; then SQ counters of the c2 decode chain (k_decode_lean).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05y}; mkdir -p $o
C2="python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 5 --warmup 2 --decode-reps 3"
for r in 1 2 3; do
  timeout -k 10 200 $C2 > $o/c2_new$r.json 2> $o/c2_new$r.err || exit 3
  LAC_LIB=tools/_probe/liblac_base.so timeout -k 10 200 $C2 > $o/c2_base$r.json 2> $o/c2_base$r.err || exit 3
done
for s in 64 256; do
  for v in new base; do
    L=""; [ $v = base ] && L=tools/_probe/liblac_base.so
    LAC_LIB=$L timeout -k 10 200 python3 bench.py --cpu-baseline off --streams $s --tokens 1024 --steps 5 --warmup 2 --decode-reps 3 > $o/b${s}_$v.json 2> $o/b${s}_$v.err || exit 3
  done
done
for f in $o/c2_*.json $o/b*_*.json; do python3 -c "
import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); p=d['parity']
print('$f'.split('/')[-1], 'enc %.3f M sym/s' % (d['value']/1e6), 'ms/step %.4f' % d['ms_per_step'], 'dec', p.get('decode',{}).get('symbols_per_s'), 'oracle', p.get('bit_exact_vs_oracle'))"; done
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d $o/d$i -o run --output-format csv -- python3 tools/dec_phase_probe.py --one-generator > $o/d$i.log 2>&1
    rc=$?
    echo "dec pmc pass $i rc=$rc"
    [ $rc -ne 0 ] && { grep -v "^    @" $o/d$i.log | tail -5; exit 3; }
done
exit 0
