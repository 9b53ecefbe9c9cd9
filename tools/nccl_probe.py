#!/usr/bin/env python3
"""Can RCCL run several ranks on ONE GPU here?  (The gatherer's nccl branch needs
world >= 2 to post sends; the GPU boxes of this pool have one MI355X.)

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29511 tools/nccl_probe.py

Every rank binds cuda:0 and tries an all_reduce, an all_gather_into_tensor and
a batch_isend_irecv; rank 0 prints one JSON line with what worked.
"""
import json
import os
import sys
import traceback

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    res = {"world": world}
    try:
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
        res["init"] = True
        x = torch.full((4,), rank + 1, dtype=torch.int64, device="cuda:0")
        dist.all_reduce(x)
        res["all_reduce"] = x.tolist()
        out = torch.empty(world, dtype=torch.int64, device="cuda:0")
        dist.all_gather_into_tensor(out, torch.tensor([rank * 10], dtype=torch.int64, device="cuda:0"))
        res["all_gather"] = out.tolist()
        # a rank sending to itself inside one batch (NCCL group semantics): the
        # gatherer's root share can then take the same P2P path as every rank's
        sb = torch.arange(16, dtype=torch.uint8, device="cuda:0") + rank
        rb = torch.zeros(16, dtype=torch.uint8, device="cuda:0")
        try:
            for w in dist.batch_isend_irecv([dist.P2POp(dist.irecv, rb, rank), dist.P2POp(dist.isend, sb, rank)]):
                w.wait()
            torch.cuda.synchronize()
            res["self_p2p"] = bool(torch.equal(rb, sb))
        except Exception as e:
            res["self_p2p"] = f"{type(e).__name__}: {e}"
        if world > 1:
            ops = []
            buf = torch.empty(16, dtype=torch.uint8, device="cuda:0")
            if rank == 0:
                ops = [dist.P2POp(dist.irecv, buf, 1)]
            elif rank == 1:
                buf.fill_(7)
                ops = [dist.P2POp(dist.isend, buf, 0)]
            if ops:
                for w in dist.batch_isend_irecv(ops):
                    w.wait()
            torch.cuda.synchronize()
            res["p2p"] = buf.tolist() if rank == 0 else "sent"
        dist.barrier()
    except Exception as e:                       # report, do not hang the box
        res["error"] = f"{type(e).__name__}: {e}"
        traceback.print_exc()
    if rank == 0:
        print(json.dumps(res), flush=True)
    try:
        dist.destroy_process_group()
    except Exception:
        pass
    return 0 if "error" not in res else 1


if __name__ == "__main__":
    sys.exit(main())
