#!/bin/bash
# Round 5: the batched gather (outboxes, device-chained pack, host-side sizes): GPU
# tests, same-box A/B against the plain headline, a kernel + HIP trace of the gather
# bench, and the 2-rank gloo rehearsal through bench.py --gpus 2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05b}; mkdir -p $o
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_dist.py tests/test_gpu_checkpoint.py tests/test_gpu_api.py -k "dist or rccl or pack or checkpoint or llama" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $o/t.log 2>&1
rc=$?; tail -3 $o/t.log; [ $rc -eq 0 ] || exit 3
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --gather --steps 40 --warmup 5 --cpu-baseline off > $o/gather$r.json 2> $o/gather$r.err || exit 3
  timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --cpu-baseline off > $o/plain$r.json 2> $o/plain$r.err || exit 3
done
python3 tools/sessions/ab/summ.py $o
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats -d $o/trace -o run --output-format csv -- python3 bench.py --gather --steps 20 --warmup 3 --cpu-baseline off > $o/trace.log 2>&1 || exit 3
LAC_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 10 --warmup 2 > $o/gloo2.json 2> $o/gloo2.err || exit 3
cat $o/gloo2.json
