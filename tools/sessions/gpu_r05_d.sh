#!/bin/bash
# Round 5: the gather with job slots (set_output) and side-stream batch packs: GPU
# dist tests, same-box A/B against the plain headline (x3), kernel trace of the
# gather bench, gloo 2-rank rehearsal.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05d}; mkdir -p $o
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_dist.py tests/test_gpu_checkpoint.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $o/t.log 2>&1
rc=$?; tail -3 $o/t.log; [ $rc -eq 0 ] || exit 3
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --gather --steps 40 --warmup 5 --cpu-baseline off > $o/gather$r.json 2> $o/gather$r.err || exit 3
  timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --cpu-baseline off > $o/plain$r.json 2> $o/plain$r.err || exit 3
done
python3 tools/sessions/ab/summ.py $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/trace -o run --output-format csv -- python3 bench.py --gather --steps 20 --warmup 3 --cpu-baseline off > $o/trace.log 2>&1 || exit 3
LAC_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 10 --warmup 2 > $o/gloo2.txt 2> $o/gloo2.err || exit 3
tail -1 $o/gloo2.txt
