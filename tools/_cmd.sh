set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -rf -x --timeout 180 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; tail -3 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --cpu-baseline off > gpurun_out/bench_$i.json 2> gpurun_out/bench_$i.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/bench_$i.json'));print('$i', d['value']/1e6, d['roofline']['kernel_ms_per_launch'], d['parity']['decode'])"
done
timeout -k 10 300 python3 bench.py --cpu-baseline off --vocab 128256 --tokens 4 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/bench_c4.json'));print('c4', d['value']/1e6, d['roofline']['frac'], d['parity']['decode'])"
