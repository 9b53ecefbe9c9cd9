"""Stream sharding across GPUs and the one exchange step: gathering bitstreams.

Streams are independent (no coder state crosses streams), so each rank owns a
contiguous block of streams, ``[r*B, (r+1)*B)``, and encodes it with no
collective at all.  The only exchange is collecting the variable-length
bitstreams afterwards: RCCL has no gather-v, so ranks
first agree on the widest stream (an all-reduce MAX of one int64) and then
all-gather fixed-width slots of that width plus the per-stream bit counts.
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
