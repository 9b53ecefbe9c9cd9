"""Deterministic, integer-only synthetic frequency tables and symbol streams.

Tables are built from splitmix64 so that every consumer (the golden-vector
generator that drives the reference coder, the CPU oracle, the GPU parity
tests) regenerates the *same* integer rows bit-for-bit from a few parameters
instead of shipping megabytes of fixtures.

Nothing here touches the coder; it only produces the integer-quantised
probability vectors that the reference's predictor protocol hands to the coder
(``CDFPredictor.dist`` is the running sum of such a row,
/root/reference/arith_code.py:76-82, 117-123).

Row kinds
---------
``loguniform``  pmf_i = (1 + (r & 255)) << ((r >> 8) % E): a 2^E-wide dynamic
                range, every entry positive.
``zeros``       as loguniform, but about 1/8 of the entries are 0.
``peaked``      a few large entries over a floor of tiny ones (LLM-like).
``flat``        pmf_i = 1 + (r % 4).
``llama64``     u64 rows at the 2^60 scale of llama_compress.py:29
                (``max(2, p*2^60)``), built from integers: big head, floor 2.
"""
from __future__ import annotations

import numpy as np

MASK64 = (1 << 64) - 1
_GOLD = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(x):
    """splitmix64 finaliser over a uint64 numpy array (wrapping arithmetic)."""
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + _GOLD
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def splitmix64_int(x: int) -> int:
    """Scalar Python-int splitmix64 (same function as :func:`splitmix64`)."""
    z = (x + 0x9E3779B97F4A7C15) & MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return z ^ (z >> 31)


def row_key(seed: int, step: int, stream: int) -> int:
    return splitmix64_int(splitmix64_int(seed & MASK64) ^ ((step * 0x100000001B3 + stream) & MASK64))


def pmf_row(seed: int, step: int, stream: int, V: int, kind: str = "loguniform",
            exp_range: int = 24) -> np.ndarray:
    """One integer pmf row of length V (uint32 unless kind == 'llama64')."""
    key = row_key(seed, step, stream)
    r = splitmix64(np.uint64(key) + np.arange(V, dtype=np.uint64))
    if kind == "loguniform" or kind == "zeros":
        mant = (r & np.uint64(255)) + np.uint64(1)
        ex = (r >> np.uint64(8)) % np.uint64(exp_range)
        p = mant << ex
        if kind == "zeros":
            p = np.where((r >> np.uint64(61)) == np.uint64(0), np.uint64(0), p)
            if not p.any():
                p[0] = 1
        return p.astype(np.uint32) if exp_range <= 24 else p
    if kind == "peaked":
        base = (r & np.uint64(3)) + np.uint64(1)
        big = ((r >> np.uint64(8)) & np.uint64(0xFFFFFF)) + np.uint64(1)
        hot = (r >> np.uint64(56)) < np.uint64(3)       # ~1.2% hot entries
        return np.where(hot, big << np.uint64(6), base).astype(np.uint32)
    if kind == "flat":
        return ((r % np.uint64(4)) + np.uint64(1)).astype(np.uint32)
    if kind == "llama64":
        hot = (r >> np.uint64(54)) < np.uint64(4)       # ~0.4% hot entries
        big = (r & np.uint64((1 << 52) - 1)) + np.uint64(1 << 40)
        p = np.where(hot, big, np.uint64(2))
        return p.astype(np.uint64)
    raise ValueError(f"unknown row kind {kind!r}")


def sample_symbol(pmf: np.ndarray, seed: int, step: int, stream: int) -> int:
    """Inverse-CDF sample with an integer uniform: bisect_right(cdf, u mod T)."""
    r = splitmix64_int(row_key(seed ^ 0x5EED, step, stream))
    if pmf.dtype == np.uint64:          # exact Python ints: the sum may pass 2^63
        import bisect
        import itertools
        cdf = list(itertools.accumulate(int(x) for x in pmf))
        return bisect.bisect_right(cdf, r % cdf[-1])
    cdf = np.cumsum(pmf, dtype=np.uint64)
    return int(np.searchsorted(cdf, np.uint64(r % int(cdf[-1])), side="right"))


def make_batch(seed: int, steps: int, streams: int, V: int, kind: str = "loguniform",
               exp_range: int = 24, sym_mode: str = "sample"):
    """pmf[steps][streams][V] and sym[steps][streams] (int32).

    ``sym_mode`` 'sample' draws each symbol from its own row (never a zero
    entry); 'uniform' draws uniformly from [0, V) (may hit zero entries).
    """
    dt = np.uint64 if (kind == "llama64" or exp_range > 24) else np.uint32
    pmf = np.empty((steps, streams, V), dtype=dt)
    sym = np.empty((steps, streams), dtype=np.int32)
    for t in range(steps):
        for b in range(streams):
            row = pmf_row(seed, t, b, V, kind, exp_range)
            pmf[t, b] = row
            if sym_mode == "sample":
                sym[t, b] = sample_symbol(row, seed, t, b)
            else:
                sym[t, b] = splitmix64_int(row_key(seed ^ 0xABC, t, b)) % V
    return pmf, sym


# ----------------------------------------------------------- device tables
def softmax_tables(steps: int, streams: int, V: int, seed: int = 1234, device="cuda",
                   sigma: float = 3.0, scale_bits: int = 31, out=None, storage_bits: int | None = None):
    """Random-logit tables on the GPU (the BASELINE.json workload).

    Per step t: logits = sigma * N(0, 1) from ``torch.Generator(device)`` seeded
    ``seed + t``; pmf = max(1, floor(softmax * 2^scale_bits)) (scale_bits <= 31 ->
    uint32 bit patterns in int32 storage, else int64 for the 2^60 llama scale of
    llama_compress.py:29 with floor 2); symbols by inverse CDF of a seeded uniform.
    ``storage_bits`` (default: 64 above scale 31) picks int64 / int32 storage.
    Returns (pmf [steps, streams, V], sym int32 [steps, streams]).
    """
    import torch
    wide = (storage_bits or (64 if scale_bits > 31 else 32)) == 64
    dt = torch.int64 if wide else torch.int32
    if out is None:
        out = torch.empty((steps, streams, V), dtype=dt, device=device)
    sym = torch.empty((steps, streams), dtype=torch.int32, device=device)
    floor_v = 2 if scale_bits >= 60 else 1
    # one generator, reseeded per step: the same streams as a fresh generator per step
    # (tests/test_gpu_api.py), without thousands of device generators (4096 of them
    # crashed torch.randn on the host under rocprofv3 --pmc, round 5)
    g = torch.Generator(device=device)
    for t in range(steps):
        g.manual_seed(seed + t)
        logits = torch.randn((streams, V), generator=g, device=device, dtype=torch.float32) * sigma
        p = torch.softmax(logits.double(), dim=-1)
        del logits
        q = torch.clamp(torch.floor(p * float(1 << scale_bits)), min=floor_v).to(torch.int64)
        del p
        cdf = torch.cumsum(q, dim=-1)
        tot = cdf[:, -1]
        u = torch.rand((streams,), generator=g, device=device, dtype=torch.float64)
        target = torch.minimum((u * tot.double()).floor().long(), tot - 1)
        sym[t] = torch.searchsorted(cdf, target.unsqueeze(1), right=True).squeeze(1).to(torch.int32)
        out[t] = q.to(dt)
        del q, cdf
    return out, sym


def logits_batch(steps: int, streams: int, V: int, seed: int = 1234, device="cuda", dtype=None,
                 sigma: float = 3.0, quantise=None):
    """Random logits [steps, streams, V] (bf16 or f32) on the GPU and symbols
    drawn from their q1 tables (``quantise`` = BatchCoder.quantize_logits) by
    inverse CDF of a seeded uniform.  Returns (logits, sym int32 [steps, streams])."""
    import torch
    dtype = dtype or torch.bfloat16
    out = torch.empty((steps, streams, V), dtype=dtype, device=device)
    sym = torch.empty((steps, streams), dtype=torch.int32, device=device)
    g = torch.Generator(device=device)                         # (reseeded per step, as above)
    for t in range(steps):
        g.manual_seed(seed + t)
        out[t] = (torch.randn((streams, V), generator=g, device=device, dtype=torch.float32) * sigma).to(dtype)
        q = quantise(out[t:t + 1])[0].to(torch.int64) & 0xFFFFFFFF
        cdf = torch.cumsum(q, dim=-1)
        del q
        tot = cdf[:, -1]
        u = torch.rand((streams,), generator=g, device=device, dtype=torch.float64)
        target = torch.minimum((u * tot.double()).floor().long(), tot - 1)
        sym[t] = torch.searchsorted(cdf, target.unsqueeze(1), right=True).squeeze(1).to(torch.int32)
        del cdf
    return out, sym
