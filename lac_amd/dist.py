"""Stream sharding across GPUs and the one exchange step: gathering bitstreams.

Streams are independent (no coder state crosses streams), so each rank owns a
contiguous block of streams, ``[r*B, (r+1)*B)``, and encodes it with no
collective at all.  The only exchange is collecting the variable-length
bitstreams on one rank.

The path bench.py times is ``BitstreamGatherer``: jobs are encoded straight into
job slots, a whole batch of them is packed by one kernel on a side stream, the
packed lengths travel between hosts (gloo), and one grouped exact-size send/recv
per batch moves every rank's packed bytes point to point to the root (RCCL over
xGMI under ``nccl``; host copies under ``gloo``).  No all-gather and no padding.

``gather_bitstreams`` is the one-off helper (an all-reduce MAX of the widest
stream, then an all-gather of fixed-width slots and the bit counts), and decoding
reverses the exchange with ``scatter_bitstreams``, which hands each rank its
shard of a job's bitstreams from the rank that holds them.
"""
from __future__ import annotations

import collections
import os
import time


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


def bitstreams_equal(got_bits, got_nbits, bits, nbits):
    """Whether an unpacked (zero padded) job ``got_*`` holds the streams ``bits`` /
    ``nbits`` (rows of a coder's output, any stride): equal bit counts, equal bytes over
    each stream's ceil(nbits/8) bytes -- past them a coder's output words hold whatever
    the buffer held before, never read and never sent -- and zeros after them in ``got``."""
    import torch
    got_bits, got_nbits = got_bits.to(bits.device), got_nbits.to(nbits.device)
    if got_bits.shape[0] != bits.shape[0] or not torch.equal(got_nbits, nbits.to(got_nbits.dtype)):
        return False
    nbytes = (nbits.to(torch.int64) + 7) // 8
    if bool((nbytes > min(got_bits.shape[1], bits.shape[1])).any()):
        return False
    w = min(got_bits.shape[1], bits.shape[1])
    live = torch.arange(got_bits.shape[1], device=bits.device)[None, :] < nbytes[:, None]
    ref = torch.zeros_like(got_bits)
    ref[:, :w] = bits[:, :w]
    return bool(torch.equal(torch.where(live, ref, torch.zeros_like(ref)), got_bits))


class HostWords:
    """``n`` int64 words of pinned host memory mapped into the device (liblac's
    lac_host_alloc, coherent): kernels write them at ``dev_addr(i)``, the host reads
    ``self[i]`` once the writing launch has completed -- no copy launch."""

    def __init__(self, lib, n):
        import ctypes as C
        self.lib, self.n = lib, int(n)
        h, d = C.c_void_p(), C.c_void_p()
        from ._lib import check
        check(lib.lac_host_alloc(8 * self.n, C.byref(h), C.byref(d)))
        self._h, self._d = h.value, d.value
        self.words = (C.c_uint64 * self.n).from_address(self._h)

    def dev_addr(self, i):
        return self._d + 8 * int(i)

    def __getitem__(self, i):
        return int(self.words[i])

    def close(self):
        """Free the words (call while the HIP runtime is up: there is no finaliser, since one
        running at interpreter exit could call into a runtime already torn down)."""
        if self._h:
            self.lib.lac_host_free(self._h)
            self._h = self._d = None


_HOST_GROUPS = {}


def host_group(group=None):
    """A gloo group over the ranks of ``group`` (default: the whole world) for the
    gatherer's host-side size exchange, made once per rank set.  ``dist.new_group`` is
    collective over the default group: every rank of the default world calls this in
    the same order."""
    import torch.distributed as dist
    ranks = tuple(dist.get_process_group_ranks(group)) if group is not None else tuple(range(dist.get_world_size()))
    world = dist.group.WORLD
    hit = _HOST_GROUPS.get(ranks)
    if hit is None or hit[0] is not world:                   # (a re-initialised world: make it again)
        hit = _HOST_GROUPS[ranks] = (world, dist.new_group(ranks=list(ranks), backend="gloo"))
    return hit[1]


class BitstreamGatherer:
    """Bitstreams of back-to-back compression jobs gathered to one rank, sized to
    the payload, in batches of jobs (the path's one exchange).

    Nothing runs on the encode's stream per job.  A BatchCoder encodes each job
    straight into a job *slot* (plane A + bit counts, ``BatchCoder.set_output``;
    ``batch`` slots per *box*, ``depth`` boxes in rotation), so a job's output needs
    no copy.  When a box fills, a side stream -- once the batch's last encode is done
    -- packs its jobs back to back into the box's outbox (one ``lac_pack_jobs`` launch
    per batch: per job a header of bit counts, 2 bytes per stream when the coder's capacity is
    below 2^16 bits, else 4, then each stream's bytes; the kernel chains the offsets in
    device memory and writes each job's packed length into pinned, device-mapped host
    words), concurrently with the next encodes.  ``lag`` jobs later (the same job
    count on every rank, so the host exchange below is a well-ordered collective), the
    host waits for the pack, reads the lengths, exchanges them with every rank over a gloo group (job
    count, streams, slot width, header size and each job's length per rank; no GPU
    work) and posts one grouped send/recv batch on the side stream: every rank sends
    exactly its packed bytes to ``root``, which receives them (RCCL over xGMI under
    nccl; the root's own share as a send to itself in the same batch, ``self_p2p``, so
    a one-rank group runs every line of the path; gloo has no self-pair, the root
    copies its share).  A box is refilled only after its pack (the encode's stream
    waits for that event, long past) and its exchange (the side stream waits).

    The round-4 form put a pack, a size all-gather, two copies and a send/recv on the
    encode's hardware queue per job, with cross-stream waits between them: ~80 us per
    1.2 ms job at world 1; packing per job on the encode's stream still cost ~16 us
    (profiles/r05/gather/).

    On the root, ``finished_jobs`` lists the jobs of the finished batches still held
    (``last_job`` the newest) and ``last_unpacked(job)`` returns one of them as (bits
    [sum of streams, width], nbits).  A batch is finished when its box is refilled or
    by ``drain``; after ``drain`` the coder presents its last job's output again (its
    slot) and later jobs continue the rotation (the next job's output is then moved to
    its place: one copy per drain).  ``bytes_sent`` / ``payload_bytes``
    count what crossed the links (the other ranks' packed jobs) and the encoded bytes
    themselves; ``meta_bytes`` what the host exchange carried.

    Coders without ``set_output`` (tests' CPU stand-ins) are copied and packed on the
    host side at ``submit``; under ``gloo`` (CPU tests, one-GPU rehearsals) the sends
    move host copies.
    """

    META = 4                                                 # int64 per rank ahead of the lengths

    def __init__(self, coder, group=None, batch: int = 8, depth: int = 3, root: int = 0, self_p2p=None,
                 lag=None, meta_group=None):
        import torch
        import torch.distributed as dist
        self.coder, self.group, self.root = coder, group, int(root)
        self.batch, self.depth = max(1, int(batch)), max(2, int(depth))
        # a batch is exchanged `lag` jobs after it closed (default: one batch later).  The
        # host waits there for the batch's pack, i.e. until the GPU has reached that
        # batch's last job; the host, which runs ahead, then still has `lag` jobs queued
        # behind it -- a lag of 2 left ~2.4 ms of queued work, and the host's exchange
        # (sizes over gloo, posting the sends) sometimes took longer: the GPU idled
        # (LAC_GATHER_TRACE, profiles/r05/gather/)
        self.lag = self.batch if lag is None else max(1, int(lag))
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.gloo = dist.get_backend(group) == "gloo"
        self.self_p2p = (not self.gloo) if self_p2p is None else bool(self_p2p)
        # sizes travel between hosts, never through the GPU: the group itself under
        # gloo, else ``meta_group`` (a gloo group over the same ranks) or one made here.
        # dist.new_group is collective over the whole default group, so without a
        # meta_group every rank of the default world constructs the gatherer (ranks
        # outside ``group`` too); the group is made once per rank set and reused.
        if self.gloo:
            self.meta_group = group
        elif meta_group is not None:
            self.meta_group = meta_group
        else:
            self.meta_group = host_group(group)
        self.width = coder.bits_stride()                      # cap_words * 8 bytes per stream
        self.hdr = 2 if self.width * 8 < (1 << 16) else 4
        B, dev = coder.streams, coder.device
        self.B, self.device = B, torch.device(dev)
        self.job_cap = B * self.hdr + B * self.width
        self.box_cap = self.batch * self.job_cap
        self.cuda = self.device.type == "cuda"
        self.native = hasattr(coder, "set_output") and self.cuda
        self.io_dev = torch.device("cpu") if self.gloo else self.device
        # the side stream at high priority: a hardware queue of its own, so its packs and
        # waits never sit between two encodes in the encode's queue (at the default
        # priority it shared that queue: profiles/r05/gather/)
        self.side = torch.cuda.Stream(device=self.device, priority=-1) if self.cuda else None
        self.boxes = []
        for _ in range(self.depth):
            bx = {"buf": torch.empty(max(self.box_cap, 1), dtype=torch.uint8, device=self.device),
                  "jobs": [], "lens": [0] * self.batch, "ends": None, "ev": None, "works": None, "meta": None,
                  "seq": 0, "closed": False}
            if self.native:
                bx["ends"] = torch.zeros(self.batch, dtype=torch.int64, device=self.device)
                bx["lens"] = HostWords(coder.lib, self.batch)
            self.boxes.append(bx)
        self.slots = None
        if self.native:                                          # per box: [job] plane A rows, bit counts
            self.words = coder.output_words()
            self.slots = [(torch.empty((self.batch, self.words), dtype=torch.int64, device=self.device),
                           torch.zeros((self.batch, B), dtype=torch.int64, device=self.device))
                          for _ in range(self.depth)]
            coder.set_output(*self._slot(0, 0))
        # root: per box and rank a receive buffer, (re)sized to the largest batch seen
        self.recv = [[None] * self.world if self.rank == self.root else None for _ in range(self.depth)]
        self.queue = collections.deque()                         # (box, job count it is exchanged at)
        self.cur = 0
        self.resume = None                                       # after drain: the slot the coder shows
        self.last_slot = None                                    # where the last job's output lives
        self.seq = 0
        self.k = 0
        self.last = None
        self.last_job = 0
        self.finished_jobs = []
        self.recent = collections.deque(maxlen=self.depth)       # root: finished batches still held
        self.bytes_sent = 0
        self.payload_bytes = 0
        self.meta_bytes = 0
        self.jobs = 0
        # LAC_GATHER_TRACE=<file>: host timestamps of every submit / exchange phase (JSON
        # lines at close), to attribute host waits (tools/sessions, profiles/r05/gather/)
        self.trace_path = os.environ.get("LAC_GATHER_TRACE")
        self.trace = [] if self.trace_path else None

    def _t(self, what, *extra):
        if self.trace is not None:
            self.trace.append((time.perf_counter(), self.k, what, *extra))

    # -- per job
    def submit(self):
        """Record the coder's just-finished job (counting from 1) in the current batch;
        exchanges whatever batch is due; points the coder at the next job's slot."""
        import torch
        self.k += 1
        self._t("submit")
        i = self.cur
        bx = self.boxes[i]
        if not self.native and bx["closed"]:
            self._prepare(i)
        n = len(bx["jobs"])
        if self.native:
            if self.resume is not None:                          # the job went to the slot drain() showed:
                li, ln = self.resume                             # move it into place (once per drain)
                if (li, ln) != (i, n):
                    for dst, src in zip(self._slot(i, n), self._slot(li, ln)):
                        dst.copy_(src)
                self.resume = None
            self.last_slot = (i, n)
        else:                                                    # any coder with the copy accessors
            bits = torch.empty((self.B, self.width), dtype=torch.uint8, device=self.device)
            nbits = torch.empty((self.B,), dtype=torch.int64, device=self.device)
            self.coder.copy_bits_into(bits)
            self.coder.copy_nbits_into(nbits)
            payload, L = pack_bitstreams(bits, nbits, self.hdr)
            L = int(L)
            off = sum(bx["lens"][:n])
            bx["buf"][off:off + L].copy_(payload[:L])
            bx["lens"][n] = L
        bx["jobs"].append(self.k)
        # due exchanges first: the sends are posted from the side stream, and RCCL's
        # stream then waits for everything queued there -- posted after the new box's
        # pack, a send waited for that pack (behind this job's encode) and held the next
        # encode in its hardware queue (87 us, profiles/r05/gather/)
        while self.queue and self.queue[0][1] <= self.k:
            self._post(self.queue.popleft()[0])
        if len(bx["jobs"]) == self.batch:
            self._close_box(i)
        if self.native:
            self._next_output()
        return self.k

    def _close_box(self, i):
        """Box i holds its last job: pack it on the side stream, due for exchange ``lag``
        jobs from now."""
        import torch
        bx = self.boxes[i]
        if self.native:
            import ctypes as C
            from ._lib import check
            done = torch.cuda.Event()
            done.record()                                        # the batch's last encode (caller's stream)
            self.side.wait_event(done)
            planes, nbits = self.slots[i]
            check(self.coder.lib.lac_pack_jobs(self.device.index or 0, C.c_void_p(planes.data_ptr()), self.words,
                                               C.c_void_p(nbits.data_ptr()), len(bx["jobs"]), self.B,
                                               self.width // 8, C.c_void_p(bx["buf"].data_ptr()), self.box_cap,
                                               self.hdr, None, C.c_void_p(bx["ends"].data_ptr()),
                                               C.c_void_p(bx["lens"].dev_addr(0)),
                                               C.c_void_p(self.side.cuda_stream)))
            bx["ev"] = torch.cuda.Event()
            bx["ev"].record(self.side)
        bx["closed"] = True
        self.queue.append((i, self.k + self.lag))
        self.cur = (i + 1) % self.depth

    def _prepare(self, i):
        """Box i is about to be refilled: exchange it (and every box queued before it, in
        order) and finish it; the encode's stream waits for its packs."""
        import torch
        bx = self.boxes[i]
        while any(q[0] == i for q in self.queue):
            self._post(self.queue.popleft()[0])
        self._finish(i)
        if bx["ev"] is not None:
            torch.cuda.current_stream(self.device).wait_event(bx["ev"])   # its slots were packed
            bx["ev"] = None
        bx["closed"] = False

    def _next_output(self):
        """Point the coder at the next job's slot (its box prepared first if closed)."""
        i = self.cur
        if self.boxes[i]["closed"]:
            self._prepare(i)
        self.coder.set_output(*self._slot(i, len(self.boxes[i]["jobs"])))

    def _slot(self, i, n):
        planes, nbits = self.slots[i]
        return planes[n], nbits[n]

    def _recv_buffer(self, i, r, n):
        import torch
        buf = self.recv[i][r]
        if buf is None or buf.numel() < n:
            buf = self.recv[i][r] = torch.empty(max(n, self.job_cap), dtype=torch.uint8, device=self.io_dev)
        return buf

    def _post(self, i):
        """Box i's exchange: sizes over the host, then one grouped send/recv batch."""
        import torch
        import torch.distributed as dist
        bx = self.boxes[i]
        self._t("post", i)
        if bx["ev"] is not None:
            self._t("ev_ready" if bx["ev"].query() else "ev_wait", i)
            bx["ev"].synchronize()                               # its packs (side stream) only
        self._t("packed", i)
        n = len(bx["jobs"])
        lens = [bx["lens"][j] for j in range(n)]
        # a failure travels in the metadata (job count -1) and every rank raises after the
        # exchange, before any send/recv is posted: raising alone would leave the other
        # ranks waiting in the all-gather or the P2P batch
        overflow = any(v >= 1 << 63 for v in lens)
        mine = torch.zeros(self.META + self.batch, dtype=torch.int64)
        mine[:self.META] = torch.tensor([-1 if overflow else n, self.B, self.width, self.hdr])
        if not overflow:
            mine[self.META:self.META + n] = torch.tensor(lens, dtype=torch.int64)
        meta = torch.empty((self.world, self.META + self.batch), dtype=torch.int64)
        _all_gather(meta.view(-1), mine, self.meta_group, self.world)
        rows = meta.tolist()
        self._t("meta", i)
        bad = [r for r, row in enumerate(rows) if row[0] < 0]
        if bad:
            raise RuntimeError(f"a packed job did not fit its outbox on rank(s) {bad}")
        if any(row[0] != n for row in rows):
            raise RuntimeError(f"ranks disagree on the batch's job count: {[row[0] for row in rows]}")
        tot = [sum(row[self.META:self.META + n]) for row in rows]
        ops = []
        if self.rank == self.root:
            for r in range(self.world):
                if r != self.root or self.self_p2p:
                    ops.append(dist.P2POp(dist.irecv, self._recv_buffer(i, r, tot[r])[:tot[r]], r, group=self.group))
        if self.rank != self.root or self.self_p2p:
            src = bx["buf"][:tot[self.rank]]
            if self.gloo and src.is_cuda:
                src = src.cpu()
            ops.append(dist.P2POp(dist.isend, src, self.root, group=self.group))
        ctx = torch.cuda.stream(self.side) if (self.side is not None and not self.gloo) else _nullctx()
        with ctx:
            bx["works"] = dist.batch_isend_irecv(ops) if ops else []
        self._t("posted", i)
        if self.rank == self.root and not self.self_p2p:         # the root's own share: a local copy
            buf = self._recv_buffer(i, self.root, tot[self.root])
            buf[:tot[self.root]].copy_(bx["buf"][:tot[self.root]])
        bx["meta"] = rows
        self.seq += 1
        bx["seq"] = self.seq
        self.bytes_sent += sum(tot) - tot[self.root]
        self.payload_bytes += sum(tot) - sum(row[0] * row[1] * row[3] for row in rows)
        self.meta_bytes += meta.numel() * 8
        self.jobs += n

    def _finish(self, i):
        """Box i's exchange is complete for the caller's stream (the root's bytes are read
        there; and the side stream packs over the outbox only after an event recorded
        later on that stream, _close_box).  Under nccl this queues a wait on an event
        the batch's send/recv passed long ago -- once per batch."""
        bx = self.boxes[i]
        if bx["works"] is None:
            return
        for w in bx["works"]:
            w.wait()
        if self.rank == self.root:
            self.last = {"jobs": list(bx["jobs"]), "meta": bx["meta"], "bufs": list(self.recv[i])}
            self.recent.append(self.last)
            self.finished_jobs = [j for b in self.recent for j in b["jobs"]]
            self.last_job = bx["jobs"][-1]
        bx.update(jobs=[], works=None, meta=None)

    def drain(self):
        """Exchange every job submitted so far and complete every batch in flight (the
        caller's stream waits for them); the coder then shows its last job's output."""
        import torch
        i = self.cur
        if self.boxes[i]["jobs"] and not self.boxes[i]["closed"]:   # a part-filled batch
            self._close_box(i)
        while self.queue:
            self._post(self.queue.popleft()[0])
        for _, j in sorted((bx["seq"], j) for j, bx in enumerate(self.boxes) if bx["works"] is not None):
            self._finish(j)
        for bx in self.boxes:
            bx["closed"] = False
        if self.native:
            cs = torch.cuda.current_stream(self.device)
            for bx in self.boxes:
                if bx["ev"] is not None:
                    cs.wait_event(bx["ev"])
                    bx["ev"] = None
            if self.last_slot is not None:                       # the last job's slot, shown again
                self.resume = self.last_slot
                self.coder.set_output(*self._slot(*self.resume))
        return self.last

    def last_unpacked(self, job=None):
        """Root: one job of the finished batches still held (``finished_jobs``; default
        the newest), rank by rank, as (bits [streams, width], nbits [streams]) with width
        the widest rank's slot.  A batch's bytes stay until its box is exchanged again,
        so read them after the ``submit`` / ``drain`` that finished it."""
        import torch
        job = self.last_job if job is None else job
        last = next((b for b in self.recent if job in b["jobs"]), None)
        if last is None:
            raise KeyError(f"job {job} is not among the finished batches held ({self.finished_jobs})")
        q = last["jobs"].index(job)
        parts = []
        for r, row in enumerate(last["meta"]):
            off = sum(row[self.META:self.META + q])
            L = row[self.META + q]
            parts.append(unpack_bitstreams(last["bufs"][r][off:off + L], row[1], row[2], row[3]))
        W = max(p[0].shape[1] for p in parts)
        bits = [torch.nn.functional.pad(p[0], (0, W - p[0].shape[1])) for p in parts]
        return torch.cat(bits), torch.cat([p[1] for p in parts])

    def close(self):
        """Free the mapped words; the coder writes to its own buffers again.  Call it
        between jobs: lac_set_output refuses a coder that is decoding or holds an
        unfinished encode (LAC_E_STATE; BatchCoder.reset() first)."""
        if self.trace:
            import json
            with open(self.trace_path, "a") as f:
                t0 = self.trace[0][0]
                for t, k, what, *extra in self.trace:
                    f.write(json.dumps({"t_us": round((t - t0) * 1e6, 1), "job": k, "what": what, "extra": extra})
                            + "\n")
            self.trace = []
        try:
            if self.native:
                self.coder.set_output(None, None)
        finally:
            for bx in self.boxes:
                if isinstance(bx["lens"], HostWords):
                    bx["lens"].close()


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
