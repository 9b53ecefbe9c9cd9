"""Multi-rank stream sharding + bitstream gather, world_size 2 over gloo on CPU."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lac_amd.dist import BitstreamGatherer, bitstreams_equal, gather_bitstreams, scatter_bitstreams, shard_range


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


def test_bitstreams_equal_ignores_bytes_past_each_stream():
    """Rows agree over ceil(nbits/8) bytes; past them the coder's row may hold anything,
    the unpacked row must hold zeros; bit counts must agree."""
    nbits = torch.tensor([0, 5, 16, 17])
    coder = torch.randint(1, 256, (4, 8), dtype=torch.uint8)
    got = torch.zeros((4, 16), dtype=torch.uint8)
    for r, n in enumerate(nbits.tolist()):
        got[r, :(n + 7) // 8] = coder[r, :(n + 7) // 8]
    assert bitstreams_equal(got, nbits, coder, nbits)
    bad = got.clone()
    bad[2, 1] ^= 1                                      # a stream byte differs
    assert not bitstreams_equal(bad, nbits, coder, nbits)
    bad = got.clone()
    bad[1, 3] = 7                                       # padding not zero
    assert not bitstreams_equal(bad, nbits, coder, nbits)
    assert not bitstreams_equal(got, nbits + 1, coder, nbits + 1)   # bytes short of the new counts
    assert not bitstreams_equal(got, torch.tensor([0, 5, 16, 18]), coder, nbits)
    assert not bitstreams_equal(got[:3], nbits[:3], coder, nbits)


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
    """CPU stand-in for BatchCoder's output accessors (the gatherer's only
    dependency): job j of rank r is a pure function of (r, j), so the parent
    process can rebuild every rank's streams to check the root's copy."""

    def __init__(self, streams, stride, rank):
        self.streams, self.stride, self.device, self.rank = streams, stride, "cpu", rank
        self.new_job(0)

    @staticmethod
    def job_data(streams, stride, rank, j):
        g = torch.Generator().manual_seed(1000 * rank + j)
        nbits = torch.randint(0, stride * 8 + 1, (streams,), generator=g, dtype=torch.int64)
        bits = torch.randint(0, 256, (streams, stride), generator=g, dtype=torch.uint8)
        return bits, nbits

    def new_job(self, j):
        self.bits, self.nbits = self.job_data(self.streams, self.stride, self.rank, j)

    def bits_stride(self):
        return self.stride

    def copy_bits_into(self, out):
        out.copy_(self.bits[:, :out.shape[1]])

    def copy_nbits_into(self, out):
        out.copy_(self.nbits)


def _record(g, seen):
    """Root: every job of the batches finished since the last call, once."""
    for j in g.finished_jobs:
        if not seen or j > seen[-1][0]:
            b, n = g.last_unpacked(j)
            seen.append((j, b.tolist(), n.tolist()))


def _gatherer_worker(rank, world, port, q, shards, stride, jobs, batch, depth):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    coder = _FakeCoder(shards[rank], stride, rank)
    g = BitstreamGatherer(coder, batch=batch, depth=depth)
    seen, when = [], []
    for j in range(1, jobs + 1):                         # more batches than outboxes: outboxes are reused
        coder.new_job(j)
        g.submit()
        if rank == 0:
            _record(g, seen)
            when.append(g.last_job)
    g.drain()
    if rank == 0:
        _record(g, seen)
    # bench.py's check: the root's newest job against a separate all-gather of every
    # rank's current output (garbage past each stream's bytes, as a coder's slots hold)
    # (gather_bitstreams needs equal shards; uneven ones are rebuilt on the root)
    if len(set(shards)) == 1:
        ref_b, ref_n = gather_bitstreams(coder.bits, coder.nbits)
    else:
        want = [_FakeCoder.job_data(shards[r], stride, r, jobs) for r in range(world)]
        ref_b, ref_n = torch.cat([b for b, _ in want]), torch.cat([n for _, n in want])
    same = bitstreams_equal(*g.last_unpacked(), ref_b, ref_n) if rank == 0 else None
    q.put((rank, seen, g.bytes_sent, g.payload_bytes, g.jobs, g.hdr, when, same))
    dist.barrier()
    dist.destroy_process_group()


def _run_gatherer(shards, stride, jobs, batch=2, depth=2):
    world = len(shards)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gatherer_worker, args=(r, world, port, q, shards, stride, jobs, batch, depth))
          for r in range(world)]
    for p in ps:
        p.start()
    res = {r[0]: r[1:] for r in (q.get(timeout=300) for _ in range(world))}
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


def _check_root(res, shards, stride, jobs, batch=2, depth=2):
    """The root saw every job exactly once, batch by batch: a batch of `batch` jobs is
    exchanged at the submit after it filled and finished when its outbox comes round
    again (`depth` batches later) or at drain(); each job holds every rank's
    streams, bytes and bit counts, exactly."""
    seen, when = res[0][0], res[0][5]
    assert [s[0] for s in seen] == list(range(1, jobs + 1))
    assert res[0][6] is True
    for k, last in enumerate(when, start=1):             # after submitting job k: job k's batch
        done = max(0, (k - 1) // batch - depth + 1)      # reuses an outbox, finishing the batch
        assert last == done * batch, (k, last)           # that held it depth batches earlier
    for j, bits, nbits in seen:
        want = [_FakeCoder.job_data(shards[r], stride, r, j) for r in range(len(shards))]
        assert nbits == [int(x) for _, n in want for x in n]
        rows = [row for b, _ in want for row in b.tolist()]
        for row, got, n in zip(rows, bits, nbits):
            nb = (n + 7) // 8
            assert got[:nb] == row[:nb] and not any(got[nb:])   # exactly the stream's bytes


@pytest.mark.parametrize("batch,depth", [(1, 2), (2, 2), (8, 2)])
def test_bitstream_gatherer_gloo_world2(batch, depth):
    """Jobs through the payload-sized, batched gather to rank 0: the root holds every
    stream's bytes and bit count, exactly; 2-byte headers (capacity < 2^16 bits)."""
    res = _run_gatherer([3, 3], 24, 5, batch, depth)
    _check_root(res, [3, 3], 24, 5, batch, depth)
    assert res[0][4] == 2


@pytest.mark.parametrize("shards,jobs,batch,depth", [([3, 0, 5, 2], 7, 2, 2), ([1, 2, 2, 2, 2, 2, 2, 2], 6, 1, 3),
                                                     ([4096 // 8] * 8, 5, 2, 2), ([1, 2, 2, 2, 2, 2, 2, 2], 7, 3, 2)])
def test_bitstream_gatherer_gloo_world4_world8_uneven(shards, jobs, batch, depth):
    """World 4 and 8 (the c5 node), uneven shards (one rank with no streams, 15
    streams over 8 ranks), more batches than outboxes at depth 2 and 3, part-filled
    last batches: seven senders, the root's receive order, outbox reuse -- the path
    RCCL takes, minus its streams and device-mapped lengths."""
    res = _run_gatherer(shards, 40, jobs, batch, depth)
    _check_root(res, shards, 40, jobs, batch, depth)


def test_bitstream_gatherer_long_job_sized_to_payload():
    """A long job (4096 symbols x 50 bits of capacity per stream): what crosses the
    links per job stays within 1.2x the encoded bytes, where
    the fixed-width slots of round 2 moved the whole capacity to every rank."""
    stride = (4096 * 50 + 256) // 8
    res = _run_gatherer([6, 6], stride, 3, 2, 2)
    _check_root(res, [6, 6], stride, 3, 2, 2)
    sent = res[0][1]                                    # (every rank counts the whole job)
    payload = res[0][2]
    assert res[0][4] == 4 and payload > 0 and sent <= 1.2 * payload, (sent, payload)


def _scatter_worker(rank, world, port, q, total):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # a job of `total` streams (uneven shards) held by rank 0 is scattered ...
    g = torch.Generator().manual_seed(7)
    width = 24
    nbits = torch.randint(0, width * 8 + 1, (total,), generator=g, dtype=torch.int64)
    bits = torch.randint(0, 256, (total, width), generator=g, dtype=torch.uint8)
    mb, mn = scatter_bitstreams(bits if rank == 0 else None, nbits if rank == 0 else None, total_streams=total)
    # ... and an even job's shards (2 per rank) gathered back reproduce it (gather pads
    # to the widest stream of the job, so compare the bytes every stream owns)
    ev = 2 * world
    g2 = torch.Generator().manual_seed(8)
    nb2 = torch.randint(0, width * 8 + 1, (ev,), generator=g2, dtype=torch.int64)
    b2 = torch.randint(0, 256, (ev, width), generator=g2, dtype=torch.uint8)
    eb, en = scatter_bitstreams(b2 if rank == 0 else None, nb2 if rank == 0 else None)
    ab, an = gather_bitstreams(eb, en)
    q.put((rank, mb.tolist(), mn.tolist(), bits.tolist(), nbits.tolist(), ab.tolist(), an.tolist(),
           b2.tolist(), nb2.tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,total", [(2, 7), (4, 7), (8, 13), (8, 3)])
def test_scatter_bitstreams_gloo(world, total):
    """Decode-side exchange: uneven shards of a job held by rank 0 (at world 8 with
    3 streams, five ranks get none), then the gather of an even job's shards
    round-trips to the source job."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_scatter_worker, args=(r, world, port, q, total)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=300) for _ in range(world)))
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    bits, nbits = res[0][2], res[0][3]
    b2, nb2 = res[0][6], res[0][7]
    for rank in range(world):
        lo, hi = shard_range(total, rank, world)
        mb, mn = res[rank][0], res[rank][1]
        assert mn == nbits[lo:hi] and mb == bits[lo:hi]
        ab, an = res[rank][4], res[rank][5]
        assert an == nb2
        for i, n in enumerate(nb2):
            assert ab[i][:(n + 7) // 8] == b2[i][:(n + 7) // 8]
