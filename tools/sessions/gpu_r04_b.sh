#!/bin/bash
# Round 4: RCCL one-rank probe (self P2P), the new dist/drop-in GPU tests, flush +
# API tests, and a one-rank bench with the gather in the timed region.
#   gpurun -- bash tools/sessions/gpu_r04_b.sh
set -u
OUT=gpurun_out/r04b
mkdir -p $OUT
step() {            # step <name> <seconds> <command...>
    local name=$1 secs=$2
    shift 2
    echo "== $name" >&2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a $OUT/status.txt >&2
    case $rc in 124|137|134|139) echo "stopping after $name" >&2; exit $rc;; esac
    return 0
}
step nccl1 200 python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 tools/nccl_probe.py
step tests 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_dist.py tests/test_gpu_dropin.py tests/test_gpu_flush.py tests/test_gpu_api.py
step gather 300 python bench.py --gather --steps 10 --warmup 2 --cpu-baseline off
tail -n 3 $OUT/*.log
