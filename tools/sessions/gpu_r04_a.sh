#!/bin/bash
# Round 4, first GPU session: RCCL probe (1 and 2 ranks on one GPU), the
# drop-in / flush / API GPU tests, the drop-in speed bench.
#   gpurun -- bash tools/sessions/gpu_r04_a.sh
# Each GPU step has its own time limit; a timeout, abort or crash stops the script.
set -u
OUT=gpurun_out/r04a
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
step nccl2 200 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 tools/nccl_probe.py
step tests 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_dropin.py tests/test_gpu_flush.py tests/test_gpu_api.py
step dropin 300 python tools/dropin_bench.py --out $OUT/dropin.json
tail -n 3 $OUT/*.log
