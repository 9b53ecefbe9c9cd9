set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/s2
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -x -rf --durations=8 --timeout 60 --timeout-method thread > gpurun_out/s2/tests.log 2>&1; rc=$?; tail -3 gpurun_out/s2/tests.log; [ $rc -ne 0 ] && exit $rc
for a in "--streams 1 --tokens 256" "--streams 1 --tokens 4096" "--streams 16 --tokens 64" "--streams 256 --tokens 32"; do
  n=$(echo $a | tr -d ' -'); timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --cpu-baseline off $a > gpurun_out/s2/b_$n.json 2>/dev/null || exit 3
done
timeout -k 10 300 python3 bench.py --cpu-baseline off > gpurun_out/s2/b_c3.json 2>/dev/null || exit 4
timeout -k 10 300 python3 bench.py --cpu-baseline off --input logits-bf16 > gpurun_out/s2/b_bf16.json 2>/dev/null || exit 5
echo done
