#!/bin/bash
# GPU session for gpurun: each GPU step has its own time limit; any abort, signal
# or timeout ends the session (pytest's ordinary failure code 1 does not).
#   tools/sessions/gpu_session.sh "<steps>"   steps: smoke tests bench prof pmc (space separated)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${1:-smoke tests bench prof}"
BENCH_ARGS="${BENCH_ARGS:-}"
run() {                       # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 25 "gpurun_out/$name.log"
    return $rc
}
ok_or_stop() {                # 0 ok; 1 = test failures (continue); anything else stops
    local rc=$1
    if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "== stopping after rc=$rc"; exit "$rc"; fi
}
for s in $STEPS; do
  case $s in
    smoke) run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"; rc=$?; [ $rc -ne 0 ] && exit $rc ;;
    tests) run tests 900 python3 -u -m pytest tests -m gpu -q -rf --timeout 180 --timeout-method thread; ok_or_stop $? ;;
    bench) run bench 600 python3 bench.py $BENCH_ARGS; ok_or_stop $? ;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
               python3 bench.py --steps 10 --warmup 2 --cpu-baseline off $BENCH_ARGS; ok_or_stop $? ;;
    pmc)   run pmc 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc -o run --output-format csv -- \
               python3 bench.py --steps 3 --warmup 1 --cpu-baseline off $BENCH_ARGS; ok_or_stop $? ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "== session done"
