"""Multi-rank stream sharding + bitstream gather, world_size 2 over gloo on CPU."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lac_amd.dist import BitstreamGatherer, gather_bitstreams, scatter_bitstreams, shard_range


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


class _FakeCoder:
    """CPU stand-in for BatchCoder's output accessors (the gatherer's only dependency)."""

    def __init__(self, streams, stride, seed):
        self.streams, self.stride, self.device = streams, stride, "cpu"
        self.g = torch.Generator().manual_seed(seed)
        self.new_job()

    def new_job(self):
        self.nbits = torch.randint(0, self.stride * 8 + 1, (self.streams,), generator=self.g, dtype=torch.int64)
        self.bits = torch.randint(0, 256, (self.streams, self.stride), generator=self.g, dtype=torch.uint8)

    def bits_stride(self):
        return self.stride

    def copy_bits_into(self, out):
        out.copy_(self.bits[:, :out.shape[1]])

    def copy_nbits_into(self, out):
        out.copy_(self.nbits)


def _gatherer_worker(rank, world, port, q, streams, stride, jobs):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    coder = _FakeCoder(streams, stride, seed=100 + rank)
    g = BitstreamGatherer(coder, depth=2)
    out = []
    for _ in range(jobs):                               # more jobs than slots: slots are reused
        coder.new_job()
        g.submit()
        got = g.last_unpacked() if rank == 0 else None
        out.append((coder.bits.tolist(), coder.nbits.tolist(),
                    None if got is None else (got[0].tolist(), got[1].tolist())))
    g.drain()
    q.put((rank, out, g.bytes_sent, g.payload_bytes, g.jobs, g.hdr))
    dist.barrier()
    dist.destroy_process_group()


def _run_gatherer(streams, stride, jobs):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gatherer_worker, args=(r, 2, port, q, streams, stride, jobs)) for r in range(2)]
    for p in ps:
        p.start()
    res = {r[0]: r[1:] for r in (q.get(timeout=180) for _ in range(2))}
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _check_root(res, jobs):
    for j in range(jobs):
        b0, n0, got = res[0][0][j]
        b1, n1, _ = res[1][0][j]
        bits, nbits = got
        assert nbits == n0 + n1                          # the root holds every stream's bit count
        for row, want, n in zip(bits, b0 + b1, n0 + n1):
            nb = (n + 7) // 8
            assert row[:nb] == want[:nb] and not any(row[nb:])   # exactly the stream's bytes


def test_bitstream_gatherer_gloo_world2():
    """Jobs through the payload-sized gather to rank 0: the root holds every
    stream's bytes and bit count, exactly; 2-byte headers (capacity < 2^16 bits)."""
    res = _run_gatherer(3, 24, 5)
    _check_root(res, 5)
    assert res[0][4] == 2


def test_bitstream_gatherer_long_job_sized_to_payload():
    """A long job (4096 symbols x 50 bits of capacity per stream): what crosses the
    links per job stays within 1.2x the encoded bytes, where
    the fixed-width slots of round 2 moved the whole capacity to every rank."""
    stride = (4096 * 50 + 256) // 8
    res = _run_gatherer(6, stride, 3)
    _check_root(res, 3)
    sent = res[0][1]                                    # (every rank counts the whole job)
    payload = res[0][2]
    assert res[0][4] == 4 and payload > 0 and sent <= 1.2 * payload, (sent, payload)


def _scatter_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # a job of 7 streams (uneven shards 3 + 4) held by rank 0 is scattered ...
    g = torch.Generator().manual_seed(7)
    total, width = 7, 24
    nbits = torch.randint(0, width * 8 + 1, (total,), generator=g, dtype=torch.int64)
    bits = torch.randint(0, 256, (total, width), generator=g, dtype=torch.uint8)
    mb, mn = scatter_bitstreams(bits if rank == 0 else None, nbits if rank == 0 else None, total_streams=total)
    # ... and an even job's shards gathered back reproduce it (gather pads to the
    # widest stream of the job, so compare the bytes every stream owns)
    eb, en = scatter_bitstreams(bits[:6] if rank == 0 else None, nbits[:6] if rank == 0 else None)
    ab, an = gather_bitstreams(eb, en)
    q.put((rank, mb.tolist(), mn.tolist(), bits.tolist(), nbits.tolist(), ab.tolist(), an.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_scatter_bitstreams_gloo_world2():
    """Decode-side exchange: uneven shards of a job held by rank 0, then the
    gather of those shards round-trips to the source job."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_scatter_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=120) for _ in range(2)))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    bits, nbits = res[0][2], res[0][3]
    for rank in (0, 1):
        lo, hi = shard_range(7, rank, 2)
        mb, mn = res[rank][0], res[rank][1]
        assert mn == nbits[lo:hi] and mb == bits[lo:hi]
        ab, an = res[rank][4], res[rank][5]
        assert an == nbits[:6]
        for i, n in enumerate(nbits[:6]):
            assert ab[i][:(n + 7) // 8] == bits[i][:(n + 7) // 8]
