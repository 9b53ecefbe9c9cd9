#!/bin/bash
# Multi-rank rehearsal: 2 ranks sharing one MI355X over gloo (the driver's 8-GPU runs use RCCL).
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/rehearse
LAC_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 6 --warmup 2 \
  > gpurun_out/rehearse/bench_2ranks_gloo.json 2> gpurun_out/rehearse/stderr.txt
rc=$?
tail -3 gpurun_out/rehearse/stderr.txt
cat gpurun_out/rehearse/bench_2ranks_gloo.json
exit $rc
