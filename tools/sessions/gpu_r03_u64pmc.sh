#!/bin/bash
# Round 3: VALU instructions per element of the u64 fine decode (SQ_INSTS_VALU pass,
# kernel trace only), round-start library vs this one, and rocprofv3 kernel stats of
# the u64 bench (decode average per launch of 16 steps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-u64pmc}; mkdir -p $o
P="python3 bench.py --pmf-bits 64 --steps 2 --warmup 1 --decode-reps 1 --cpu-baseline off"
for v in head new; do
  lib=lac_amd/liblac.so; [ $v = head ] && lib=tools/sessions/ab/liblac_r03_head.so
  LAC_LIB=$lib timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD --kernel-trace \
      -d $o/pmc_$v -o run --output-format csv -- $P > $o/pmc_$v.log 2>&1 || { tail -20 $o/pmc_$v.log; exit 3; }
  echo "pmc $v ok"
done
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $o/stats -o run --output-format csv -- \
    python3 bench.py --pmf-bits 64 --steps 10 --cpu-baseline off > $o/stats.log 2>&1 || { tail -20 $o/stats.log; exit 3; }
tail -1 $o/stats.log | cut -c1-300
python3 tools/pmc_summary.py $o/pmc_head decode_wave_fine
python3 tools/pmc_summary.py $o/pmc_new decode_wave_fine
echo "== done"
