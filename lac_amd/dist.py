"""Stream sharding across GPUs and the one exchange step: gathering bitstreams.

Streams are independent (no coder state crosses streams), so each rank owns a
contiguous block of streams, ``[r*B, (r+1)*B)``, and encodes it with no
collective at all.  The only exchange is collecting the variable-length
bitstreams afterwards: RCCL has no gather-v, so ranks
first agree on the widest stream (an all-reduce MAX of one int64) and then
all-gather fixed-width slots of that width plus the per-stream bit counts.
Decoding reverses it: ``scatter_bitstreams`` hands each rank its shard of a
job's bitstreams from the rank that holds them.
With the ``nccl`` backend (RCCL on ROCm) the tensors stay in HBM and move
over xGMI; with ``gloo`` (tests) they are CPU tensors.
"""
from __future__ import annotations


def shard_range(total_streams: int, rank: int, world: int):
    """Contiguous block of streams owned by ``rank``."""
    lo = total_streams * rank // world
    hi = total_streams * (rank + 1) // world
    return lo, hi


def gather_bitstreams(bits, nbits, group=None):
    """All-gather per-stream packed bitstreams.

    bits   uint8 tensor [B, stride] (stream b's bytes at row b, zero padded)
    nbits  int64 tensor [B] (bit counts)
    Returns (all_bits [world*B, width], all_nbits [world*B]) on every rank,
    width = max over all streams of ceil(nbits/8) rounded up to 8.
    """
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    B = bits.shape[0]
    width = ((nbits.max() + 7) // 8 if B else torch.zeros((), dtype=torch.int64, device=nbits.device)).to(torch.int64)
    width = width.reshape(1).clone()
    if width.is_cuda and dist.get_backend(group) == "gloo":
        width = width.cpu()
    dist.all_reduce(width, op=dist.ReduceOp.MAX, group=group)
    w = int(width.item())
    w = max(8, (w + 7) // 8 * 8)
    if w > bits.shape[1]:
        pad = torch.zeros((B, w - bits.shape[1]), dtype=bits.dtype, device=bits.device)
        slot = torch.cat([bits, pad], dim=1)
    else:
        slot = bits[:, :w].contiguous()
    out_bits = torch.empty((world * B, w), dtype=bits.dtype, device=bits.device)
    out_n = torch.empty((world * B,), dtype=nbits.dtype, device=nbits.device)
    _all_gather(out_bits, slot, group, world)
    _all_gather(out_n, nbits.contiguous(), group, world)
    return out_bits, out_n


def scatter_bitstreams(all_bits=None, all_nbits=None, total_streams=None, src=0, group=None, device=None):
    """Decode side of the exchange: rank ``src`` holds every
    stream's packed bits ``[total, width]`` (uint8, a gathered job or a stored
    one) and bit counts ``[total]`` (int64); every rank receives its own
    contiguous shard ``shard_range(total, rank, world)`` and decodes it
    independently (``BatchCoder.decode_open(bits, nbits)``).  Non-source ranks
    pass ``None`` for the tensors; shapes travel in one broadcast.  Shards are
    padded to the largest one so the scatter moves equal-sized slots.
    Returns ``(bits [hi - lo, width], nbits [hi - lo])`` on every rank.
    """
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    gloo = dist.get_backend(group) == "gloo"
    if rank == src:
        device = all_bits.device
    dev = torch.device("cpu") if gloo else torch.device(device if device is not None else "cuda")
    hdr = torch.zeros(2, dtype=torch.int64, device=dev)
    if rank == src:
        hdr[0], hdr[1] = all_bits.shape[0], all_bits.shape[1]
    dist.broadcast(hdr, src=src, group=group)
    total, width = int(hdr[0]), int(hdr[1])
    if total_streams is not None and total_streams != total:
        raise ValueError(f"source holds {total} streams, caller expected {total_streams}")
    S = max(hi - lo for lo, hi in (shard_range(total, r, world) for r in range(world)))
    lo, hi = shard_range(total, rank, world)
    out_b = torch.empty((S, width), dtype=torch.uint8, device=dev)
    out_n = torch.empty((S,), dtype=torch.int64, device=dev)
    sb = sn = None
    if rank == src:
        hb, hn = (all_bits.cpu(), all_nbits.cpu()) if gloo else (all_bits, all_nbits.to(torch.int64))
        sb, sn = [], []
        for r in range(world):
            a, z = shard_range(total, r, world)
            pb = torch.zeros((S, width), dtype=torch.uint8, device=hb.device)
            pn = torch.zeros((S,), dtype=torch.int64, device=hn.device)
            pb[:z - a] = hb[a:z]
            pn[:z - a] = hn[a:z]
            sb.append(pb)
            sn.append(pn)
    dist.scatter(out_b, sb, src=src, group=group)
    dist.scatter(out_n, sn, src=src, group=group)
    out_b, out_n = out_b[:hi - lo], out_n[:hi - lo]
    if gloo and device is not None and torch.device(device).type != "cpu":
        out_b, out_n = out_b.to(device), out_n.to(device)
    return out_b.contiguous(), out_n.contiguous()


def _all_gather(out, inp, group, world):
    import torch.distributed as dist
    if out.is_cuda and dist.get_backend(group) == "gloo":   # rehearsal runs: gloo moves host tensors
        host = out.cpu()
        _all_gather(host, inp.cpu(), group, world)
        out.copy_(host)
        return
    try:
        dist.all_gather_into_tensor(out, inp, group=group)
    except (RuntimeError, NotImplementedError):       # backends without the fused form
        dist.all_gather(list(out.chunk(world)), inp, group=group)


class BitstreamGatherer:
    """Fixed-width, asynchronous, double-buffered bitstream all-gather for
    back-to-back compression jobs.

    ``gather_bitstreams`` agrees on the widest stream first (an all-reduce and a
    host read), which serialises every job behind two collective latencies.  A
    job's slot width is known up front: no stream can exceed the coder's
    capacity (``cap_words`` 8-byte words).  So each ``submit()`` copies the
    packed bits and bit counts into one of ``depth`` slot buffers on the
    caller's stream and enqueues the all-gathers with ``async_op=True``: RCCL
    runs them on its own stream while the next job's encode kernel streams its
    tables, and the caller's stream only waits for a collective when its slot is
    about to be reused ``depth`` jobs later.  ``drain()`` makes the caller's
    stream wait for everything still in flight.

    Under ``gloo`` (CPU tests, one-GPU rehearsals) the gather goes through host
    tensors synchronously, like ``gather_bitstreams``.
    """

    def __init__(self, coder, group=None, depth: int = 2):
        import torch
        import torch.distributed as dist
        self.coder, self.group, self.depth = coder, group, max(1, int(depth))
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.gloo = dist.get_backend(group) == "gloo"
        self.width = coder.bits_stride()                      # cap_words * 8 bytes per stream
        B, dev = coder.streams, coder.device
        self.slots = [(torch.empty((B, self.width), dtype=torch.uint8, device=dev),
                       torch.empty((B,), dtype=torch.int64, device=dev)) for _ in range(self.depth)]
        self.outs = [(torch.empty((self.world * B, self.width), dtype=torch.uint8, device=dev),
                      torch.empty((self.world * B,), dtype=torch.int64, device=dev)) for _ in range(self.depth)]
        self.pending = [None] * self.depth
        self.k = 0
        self.last = None

    def submit(self):
        """Gather the coder's current output; returns the (bits, nbits) output
        buffers, valid on the caller's stream after ``drain()``."""
        import torch.distributed as dist
        i = self.k % self.depth
        self.k += 1
        self._wait(i)                                           # slot i's previous gather is done
        bits, nbits = self.slots[i]
        self.coder.copy_bits_into(bits)                          # on the caller's stream
        self.coder.copy_nbits_into(nbits)
        ob, on = self.outs[i]
        if self.gloo:
            _all_gather(ob, bits, self.group, self.world)
            _all_gather(on, nbits, self.group, self.world)
        else:
            self.pending[i] = [dist.all_gather_into_tensor(ob, bits, group=self.group, async_op=True),
                               dist.all_gather_into_tensor(on, nbits, group=self.group, async_op=True)]
        self.last = (ob, on)
        return self.last

    def _wait(self, i):
        if self.pending[i]:
            for w in self.pending[i]:
                w.wait()                                        # caller's stream waits; the host does not
            self.pending[i] = None

    def drain(self):
        for i in range(self.depth):
            self._wait(i)
        return self.last
