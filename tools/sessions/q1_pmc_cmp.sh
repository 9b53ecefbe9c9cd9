#!/bin/bash
# SQ counters: bf16 Qwen2 (V=151936, row groups, shape 20) vs bf16 c4 (V=128256, shape 15).
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/q1cmp
for cfg in "qwen:--vocab 151936" "c4:--vocab 128256"; do
  name=${cfg%%:*}; args=${cfg#*:}
  i=0
  for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/q1cmp/$name/p$i -o run --output-format csv -- \
        python3 bench.py --steps 3 --warmup 1 --cpu-baseline off --decode-reps 1 --input logits-bf16 --tokens 8 $args > gpurun_out/q1cmp/$name.p$i.log 2>&1 || exit 3
  done
  python3 tools/pmc_summary.py gpurun_out/q1cmp/$name k_q1_stats > gpurun_out/q1cmp/$name.summary.txt
done
cat gpurun_out/q1cmp/*.summary.txt
