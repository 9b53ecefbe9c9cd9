"""Multi-rank stream sharding + bitstream gather, world_size 2 over gloo on CPU."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lac_amd.dist import gather_bitstreams, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    B = 5
    g = torch.Generator().manual_seed(rank)
    nbits = torch.randint(0, 200, (B,), generator=g, dtype=torch.int64)
    bits = torch.zeros((B, 32), dtype=torch.uint8)
    for b in range(B):
        n = (int(nbits[b]) + 7) // 8
        bits[b, :n] = torch.randint(0, 256, (n,), generator=g, dtype=torch.uint8)
    allb, alln = gather_bitstreams(bits, nbits)
    q.put((rank, bits.tolist(), nbits.tolist(), allb.tolist(), alln.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_partitions():
    for total in (1, 7, 4096, 32768):
        for world in (1, 2, 3, 8):
            rs = [shard_range(total, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == total
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))


def test_gather_bitstreams_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, b0, n0, A0, N0), (r1, b1, n1, A1, N1) = res
    assert A0 == A1 and N0 == N1 == n0 + n1
    width = len(A0[0])
    assert width % 8 == 0 and width >= max((n + 7) // 8 for n in n0 + n1)
    for i, (row, n) in enumerate(zip(b0 + b1, n0 + n1)):
        nb = (n + 7) // 8
        assert A0[i][:nb] == row[:nb]
