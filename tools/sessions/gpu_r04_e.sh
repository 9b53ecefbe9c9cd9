#!/bin/bash
# Round 4: dist GPU tests (pack kernel), gather-in-timed-region bench vs plain, bf16 Qwen2
# decode with back-to-back passes, PMC of the logits decode kernels at bf16 c3 / c4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r04e}; mkdir -p $o
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dist.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $o/t.log 2>&1
rc=$?; tail -2 $o/t.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 200 python3 bench.py --gather --steps 20 --warmup 3 --cpu-baseline off > $o/gather.json 2> $o/gather.err || exit 3
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --cpu-baseline off > $o/nogather.json 2> $o/nogather.err || exit 3
timeout -k 10 200 python3 bench.py --input logits-bf16 --vocab 151936 --steps 8 --warmup 3 --cpu-baseline off --decode-reps 5 > $o/qwen2.json 2> $o/qwen2.err || exit 3
python3 tools/sessions/ab/summ.py $o
bash tools/sessions/pmc_passes.sh ${1:-r04e}/pmc_c3 tools/q1_b2b.py --vocab 32000 --reps 3 || exit 3
bash tools/sessions/pmc_passes.sh ${1:-r04e}/pmc_c4 tools/q1_b2b.py --vocab 128256 --reps 3 || exit 3
python3 tools/pmc_summary.py $o/pmc_c3 k_q1_decode
python3 tools/pmc_summary.py $o/pmc_c4 k_q1_decode
