#!/bin/bash
# Quick GPU check of the tree: GPU tests, smoke, headline bench (any failure ends it).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-check}; mkdir -p $o; shift || true
step() {
    local name=$1 secs=$2; shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "$o/$name.out" 2> "$o/$name.err"
    local rc=$?
    echo "== $name rc=$rc"; tail -n 2 "$o/$name.out" | cut -c1-400
    [ $rc -ne 0 ] && { tail -n 20 "$o/$name.err"; exit $rc; }
    return 0
}
step tests 600 python3 -u -m pytest tests -m gpu -q -x -rf --timeout 120 --timeout-method thread
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench_c3 300 python3 bench.py
echo "== done"
