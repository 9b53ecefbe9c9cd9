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


def pack_bitstreams(bits, nbits, hdr_bytes):
    """Device-side packing, no host synchronisation: a header of every stream's bit
    count (``hdr_bytes`` = 2 or 4 bytes each, little endian) followed by the
    streams' bytes back to back (ceil(nbits/8) each).  Returns (payload, L):
    ``payload`` uint8 of the worst-case size, its first ``L`` (a 0-d device
    tensor) bytes valid."""
    import torch
    B, W = bits.shape
    dev = bits.device
    nb = nbits.to(torch.int64)
    nbytes = (nb + 7) // 8
    hdr = torch.stack([(nb >> (8 * i)) & 0xFF for i in range(hdr_bytes)], 1).to(torch.uint8).reshape(-1)
    start = B * hdr_bytes + torch.cumsum(nbytes, 0) - nbytes                 # each stream's first byte
    cap = B * hdr_bytes + B * W
    j = torch.arange(W, device=dev)
    dest = torch.where(j[None, :] < nbytes[:, None], start[:, None] + j[None, :],
                       torch.full((1, 1), cap, dtype=torch.int64, device=dev))   # the rest: one dump byte
    payload = torch.zeros(cap + 1, dtype=torch.uint8, device=dev)
    payload[:B * hdr_bytes] = hdr
    payload.scatter_(0, dest.reshape(-1), bits.reshape(-1))
    L = B * hdr_bytes + nbytes.sum()
    return payload, L


def unpack_bitstreams(payload, streams, width, hdr_bytes):
    """Inverse of pack_bitstreams -> (bits [streams, width] zero padded, nbits int64 [streams])."""
    import torch
    dev = payload.device
    h = payload[:streams * hdr_bytes].reshape(streams, hdr_bytes).to(torch.int64)
    nb = sum(h[:, i] << (8 * i) for i in range(hdr_bytes))
    nbytes = (nb + 7) // 8
    start = streams * hdr_bytes + torch.cumsum(nbytes, 0) - nbytes
    j = torch.arange(width, device=dev)
    src = torch.clamp(start[:, None] + j[None, :], max=payload.numel() - 1)
    out = torch.where(j[None, :] < nbytes[:, None], payload[src], torch.zeros((), dtype=torch.uint8, device=dev))
    return out, nb


class BitstreamGatherer:
    """Bitstreams of back-to-back compression jobs gathered to one rank, sized to
    the payload, with no host synchronisation on the GPU's path.

    Per job, on every rank (``submit``): the coder's streams are packed on the
    device into a header of bit counts (2 bytes per stream when the coder's
    capacity is below 2^16 bits, else 4) plus the streams' bytes back to back
    (``pack_bitstreams``), and four int64 -- the packed length, the rank's stream
    count, its slot width and header size -- are all-gathered, asynchronously.
    Ranks may hold different numbers of streams (uneven shards).  Under nccl the
    sizes reach the host through a pinned copy on a side stream, so the host
    waits only for this job's packing, never for the next job's encode, which it
    has already enqueued.  At the next ``submit`` (or ``drain``) every rank sends
    exactly its packed bytes to ``root`` and the root receives them (one grouped
    send/recv batch on the side stream: RCCL over xGMI), ordered after the
    packing only.  Under nccl the root's own share takes the same batch as a send
    to itself (``self_p2p``; NCCL group semantics), so a one-rank job runs every
    line of the RCCL path; gloo has no self-pair, the root copies its share.
    xGMI carries the payload, the header and 32 bytes per rank -- not a
    worst-case slot per stream, and not to every rank.

    On the root, ``last`` describes the last finished job (``last_job`` its
    number, counting from 1) and ``last_unpacked()`` returns its streams as
    (bits [sum of streams, width], nbits).  A job is finished when its slot is
    reused (``depth`` jobs later) or by ``drain``.  ``bytes_sent`` /
    ``payload_bytes`` count what crossed the links and the encoded bytes
    themselves (bench.py reports both).

    Under ``gloo`` (CPU tests, one-GPU rehearsals) the same deferred exchange runs
    on host tensors; only the streams, events and pinned copies are nccl's.
    """

    META = 4                                                 # int64 per rank: L, streams, width, hdr

    def __init__(self, coder, group=None, depth: int = 2, root: int = 0, self_p2p=None):
        import torch
        import torch.distributed as dist
        self.coder, self.group, self.depth, self.root = coder, group, max(1, int(depth)), int(root)
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.gloo = dist.get_backend(group) == "gloo"
        self.self_p2p = (not self.gloo) if self_p2p is None else bool(self_p2p)
        self.width = coder.bits_stride()                      # cap_words * 8 bytes per stream
        self.hdr = 2 if self.width * 8 < (1 << 16) else 4
        B, dev = coder.streams, coder.device
        self.B = B
        self.cap = B * self.hdr + B * self.width + 1
        self.io_dev = torch.device("cpu") if self.gloo else torch.device(dev)
        # per slot the packed payload (a BatchCoder packs its planes directly, lac_pack_bits)
        # or, for other coders, the copies pack_bitstreams works from
        if hasattr(coder, "pack_bits"):
            self.packed = [(torch.empty(self.cap, dtype=torch.uint8, device=dev),
                            torch.tensor([0, B, self.width, self.hdr], dtype=torch.int64, device=dev))
                           for _ in range(self.depth)]
            self.slots = None
        else:
            self.packed = None
            self.slots = [(torch.empty((B, self.width), dtype=torch.uint8, device=dev),
                           torch.empty((B,), dtype=torch.int64, device=dev)) for _ in range(self.depth)]
        # root: per slot and rank a receive buffer, (re)sized to the largest payload seen
        self.recv = [[None] * self.world if self.rank == self.root else None for _ in range(self.depth)]
        self.meta = [torch.empty(self.world * self.META, dtype=torch.int64, device=self.io_dev)
                     for _ in range(self.depth)]
        self.meta_host = [torch.empty(self.world * self.META, dtype=torch.int64).pin_memory()
                          if not self.gloo and torch.cuda.is_available()
                          else torch.empty(self.world * self.META, dtype=torch.int64) for _ in range(self.depth)]
        self._shape_meta = torch.tensor([B, self.width, self.hdr], dtype=torch.int64, device=dev)
        self.state = [None] * self.depth                        # per slot: dict of the job in flight
        self.side = torch.cuda.Stream(device=dev) if not self.gloo else None
        self.k = 0
        self.last = None
        self.last_job = 0
        self.bytes_sent = 0
        self.payload_bytes = 0
        self.jobs = 0

    # -- per job
    def submit(self):
        """Queue the coder's current output for the root; returns the job's slot."""
        import torch
        import torch.distributed as dist
        i = self.k % self.depth
        self.k += 1
        self._finish(i)                                         # slot i's previous job, if any
        self._send_pending()                                    # the jobs queued since: their exact sends
        if self.packed is not None:                              # BatchCoder: one pack on the device,
            payload, mine = self.packed[i]                       # its length straight into the sizes row
            self.coder.pack_bits(payload, self.hdr, mine[:1])    # (on the caller's stream)
        else:                                                    # any coder with the copy accessors
            bits, nbits = self.slots[i]
            self.coder.copy_bits_into(bits)
            self.coder.copy_nbits_into(nbits)
            payload, L = pack_bitstreams(bits, nbits, self.hdr)
            mine = torch.cat([L.to(torch.int64).reshape(1), self._shape_meta])
        st = {"payload": payload, "job": self.k}
        if self.gloo:
            _all_gather(self.meta[i], mine.cpu(), self.group, self.world)
            st["meta"] = self.meta[i].view(self.world, self.META).tolist()
            st["payload"] = payload[:st["meta"][self.rank][0]].cpu()    # the packed bytes only
            self.state[i] = st
            return i
        ev = torch.cuda.Event()
        ev.record()                                             # packing done (caller's stream)
        work = dist.all_gather_into_tensor(self.meta[i], mine, group=self.group, async_op=True)
        with torch.cuda.stream(self.side):
            self.side.wait_event(ev)
            work.wait()                                         # the side stream waits for the sizes
            self.meta_host[i].copy_(self.meta[i], non_blocking=True)
            st["meta_ready"] = torch.cuda.Event()
            st["meta_ready"].record(self.side)
        st["packed"] = ev
        self.state[i] = st
        return i

    def _send_pending(self):
        """Post the sends of every queued job, oldest first (point-to-point order
        must match between each rank and the root)."""
        for _, i in sorted((st["job"], i) for i, st in enumerate(self.state) if st is not None):
            self._send(i)

    def _recv_buffer(self, i, r, n):
        import torch
        buf = self.recv[i][r]
        if buf is None or buf.numel() < n:
            buf = self.recv[i][r] = torch.empty(max(n, self.cap), dtype=torch.uint8, device=self.io_dev)
        return buf

    def _send(self, i):
        """Post job i's exact-size send (every rank) / receives (root), once its
        sizes are on the host."""
        import torch
        import torch.distributed as dist
        st = self.state[i]
        if st is None or "works" in st:
            return
        if "meta" not in st:
            st["meta_ready"].synchronize()                      # this job's packing + size gather only
            st["meta"] = self.meta_host[i].view(self.world, self.META).tolist()
        lens = [m[0] for m in st["meta"]]
        ops = []
        if self.rank == self.root:
            for r in range(self.world):
                if r != self.root or self.self_p2p:
                    ops.append(dist.P2POp(dist.irecv, self._recv_buffer(i, r, lens[r])[:lens[r]], r,
                                          group=self.group))
        if self.rank != self.root or self.self_p2p:
            ops.append(dist.P2POp(dist.isend, st["payload"][:lens[self.rank]], self.root, group=self.group))
        ctx = torch.cuda.stream(self.side) if not self.gloo else _nullctx()
        with ctx:
            if not self.gloo:
                self.side.wait_event(st["packed"])
            st["works"] = dist.batch_isend_irecv(ops) if ops else []
        if self.rank == self.root and not self.self_p2p:        # the root's own share: a local copy
            buf = self._recv_buffer(i, self.root, lens[self.root])
            buf[:lens[self.root]].copy_(st["payload"][:lens[self.root]], non_blocking=True)
        self.bytes_sent += sum(lens) - lens[self.root] + 8 * self.META * self.world
        self.payload_bytes += sum(lens) - sum(m[1] * m[3] for m in st["meta"])
        self.jobs += 1

    def _finish(self, i):
        import torch
        st = self.state[i]
        if st is None:
            return
        self._send_pending()                                    # older jobs first, then this one
        # the caller's stream waits for this job's sends and receives only (its payload
        # slot is about to be reused; the root's received bytes are then visible) -- not
        # for the whole side stream, which already holds later jobs' size exchanges: that
        # wait cost ~60 us of cross-queue hops per job (profiles/r04/gather/)
        for w in st["works"]:
            w.wait()
        if self.rank == self.root:
            self.last = [(self.recv[i][r], m[0], m[1], m[2], m[3]) for r, m in enumerate(st["meta"])]
            self.last_job = st["job"]
        self.state[i] = None

    def drain(self):
        """Complete every job in flight (the caller's stream waits for them)."""
        self._send_pending()
        for _, j in sorted((st["job"], j) for j, st in enumerate(self.state) if st is not None):
            self._finish(j)
        return self.last

    def last_unpacked(self):
        """Root: the last finished job's streams, rank by rank, as (bits [streams,
        width], nbits [streams]) with width the widest rank's slot."""
        import torch
        parts = [unpack_bitstreams(p[:n], b, w, h) for p, n, b, w, h in self.last]
        W = max(p[0].shape[1] for p in parts)
        bits = [torch.nn.functional.pad(p[0], (0, W - p[0].shape[1])) for p in parts]
        return torch.cat(bits), torch.cat([p[1] for p in parts])


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
