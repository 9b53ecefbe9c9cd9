# final round check: GPU tests, headline bench, logits benches, rocprofv3 stats of the headline
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/fin
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -x -rf --timeout 60 --timeout-method thread > gpurun_out/fin/tests.log 2>&1; rc=$?; tail -2 gpurun_out/fin/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py > gpurun_out/fin/bench_c3.json 2>gpurun_out/fin/bench_c3.err || exit 3
timeout -k 10 300 python3 bench.py --cpu-baseline off --input logits-bf16 > gpurun_out/fin/bench_bf16.json 2>/dev/null || exit 4
timeout -k 10 300 python3 bench.py --cpu-baseline off --input logits-bf16 --vocab 128256 --steps 5 > gpurun_out/fin/bench_bf16_c4.json 2>/dev/null || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fin/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/fin/prof.json 2>/dev/null || exit 6
timeout -k 10 300 python3 bench.py --cpu-baseline off --pmf-bits 64 > gpurun_out/fin/bench_u64.json 2>/dev/null || exit 7
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin/smoke.log 2>&1 || exit 8
echo done
