"""Seeded random configurations through every encode and decode kernel.

Each case draws a vocabulary (odd sizes take the scalar-load kernels), a
precision, a row family (log-uniform, with zeros, peaked, flat, llama-scale
u64 rows that always take fudged_dist), a stream count and a step count, then
checks the GPU bytes of the split, fused and AUTO encoders against the C oracle
(oracle/lac_oracle.c, pinned to the reference's golden vectors) and decodes the
stream back with every decode kernel (per-step, one-wave fine and chunk, stats,
block).  Cases are fixed by the seed, so a failure reproduces exactly.
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from lac_amd import synth  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
KINDS = ("loguniform", "zeros", "peaked", "flat", "llama64")
DECODE_PATHS = ("split", "fused", "fused_chunk", "stats", "block")


def _case(i):
    rng = np.random.default_rng(9000 + i)
    V = int(rng.choice([2, 3, 17, 256, 999, 1000, 4096, 5003, 32000, 32004, 40000, 65537]))
    kind = KINDS[int(rng.integers(len(KINDS)))]
    lo = max(int(np.ceil(np.log2(V))) + 2, 8)
    prec = int(rng.integers(lo, 62)) if kind != "llama64" else int(rng.choice([40, 48, 61]))
    B = int(rng.integers(1, 25))
    steps = int(rng.integers(1, 13))
    while B * steps * V > 3_000_000 and B > 1:
        B //= 2
    return V, kind, prec, B, steps


N_PMF = int(os.environ.get("LAC_FUZZ_N", "36"))          # more cases: LAC_FUZZ_N=400 pytest ...
N_LOGITS = int(os.environ.get("LAC_FUZZ_LOGITS_N", "24"))


@pytest.mark.parametrize("i", range(N_PMF))
def test_fuzz_encode_decode_all_paths(i):
    from lac_amd.batch import BatchCoder
    from oracle import oracle as coracle
    V, kind, prec, B, steps = _case(i)
    pmf, sym = synth.make_batch(4242 + i, steps, B, V, kind)
    bits = 64 if pmf.dtype == np.uint64 else 32
    out, nb, status, rc = coracle.encode_batch(pmf, sym, prec, nthreads=8)
    assert rc == 0 and not status.any(), (V, kind, prec, B, steps)
    dpmf = torch.from_numpy(pmf.view(np.int64 if bits == 64 else np.int32)).to(DEV)
    dsym = torch.from_numpy(sym).to(DEV)
    c = BatchCoder(V, B, prec=prec, pmf_bits=bits, capacity_bits=steps * (prec + 2) + 256, device=DEV)
    for path in ("split", "fused", "auto"):
        c.set_path(path)
        c.encode_job(dpmf, dsym)
        data, n = c.to_bytes()
        for b in range(B):
            assert int(n[b]) == int(nb[b]), (path, b)
            assert data[b] == out[b, :(int(nb[b]) + 7) // 8].tobytes(), (path, b)
    for path in DECODE_PATHS:
        c.set_decode_path(path)
        c.decode_open()
        got = c.decode(dpmf)
        assert torch.equal(got, dsym), (path, V, kind, prec, B, steps)
    c.close()


def _logits_case(i):
    rng = np.random.default_rng(7000 + i)
    dtype = "bf16" if rng.random() < 0.6 else "f32"
    sizes = [8, 64, 1000, 4096, 8200, 32000, 32768 + 8, 65536]
    sizes += [128256, 128512, 128520, 131072] if dtype == "bf16" else [65536 - 8]
    # rows over groups of 2..4 blocks (shape 19)
    sizes += [131080, 151936, 262144, 300000] if dtype == "bf16" else [65540, 128256, 151936, 200000, 262144]
    # a whole row per 8-wave block (shape 22: <= 20480 vectors) and either side of its
    # limit (shape 23 past it)
    sizes += [147464, 163840, 163848, 202048, 208904] if dtype == "bf16" else [73732, 81920, 81924, 100280, 104456]
    V = int(rng.choice(sizes))
    lo = max(int(np.ceil(np.log2(V))) + 2, 8)
    prec = int(rng.integers(lo, 62))
    B = int(rng.integers(1, 40))
    steps = int(rng.integers(1, 9))
    while B * steps * V > 2_000_000 and B > 1:
        B //= 2
    scale = float(rng.choice([0.25, 3.0, 12.0]))
    shape = int(rng.choice([0, 0, 0] + list(range(1, 24))))
    if shape in (5, 7, 9, 11, 12, 13, 16):             # retired shapes (lac.h LAC_OPT_Q1_SHAPE): AUTO
        shape = 0
    return dtype, V, prec, B, steps, scale, shape


@pytest.mark.parametrize("i", range(N_LOGITS))
def test_fuzz_logits_encode_decode(i):
    """Seeded random logits configurations (vocab across every row-stats shape
    boundary, bf16/f32, prec, scale, NaN/inf entries, a random forced shape or
    AUTO): GPU tables, bytes and decodes equal the C oracle (q1 + encode)."""
    from lac_amd._lib import LacError
    from lac_amd.batch import BatchCoder
    from oracle import oracle as coracle
    dtype, V, prec, B, steps, scale, shape = _logits_case(i)
    rng = np.random.default_rng(100 + i)
    x = (rng.standard_normal((steps, B, V)) * scale).astype(np.float32)
    if V >= 8:
        x[0, 0, 1] = np.nan
        x[-1, -1, 2] = -np.inf
    dl = torch.from_numpy(x).to(DEV)
    dl = dl.to(torch.bfloat16) if dtype == "bf16" else dl
    host = dl.view(torch.int16).cpu().numpy().view(np.uint16) if dtype == "bf16" else dl.cpu().numpy()
    pmf = coracle.q1_quantize(host, prec)
    c = np.cumsum(pmf.astype(np.uint64), axis=-1)
    r = (rng.random((steps, B)) * c[..., -1]).astype(np.uint64)
    sym = np.empty((steps, B), dtype=np.int32)
    for idx in np.ndindex(steps, B):
        sym[idx] = min(int(np.searchsorted(c[idx], r[idx], side="right")), V - 1)
    out, nb, status, rc = coracle.encode_batch(pmf, sym, prec, nthreads=8)
    assert rc == 0 and not status.any()
    coder = BatchCoder(V, B, prec=prec, pmf_bits=32, capacity_bits=steps * (prec + 2) + 256, device=DEV)
    assert (coder.quantize_logits(dl).cpu().numpy().view(np.uint32) == pmf).all()
    if shape:
        coder.set_q1_shape(shape)
    dsym = torch.from_numpy(sym).to(DEV)
    try:
        coder.encode_logits_job(dl, dsym)
    except LacError:                                   # a forced shape that cannot hold the row
        coder.set_q1_shape(0)
        coder.encode_logits_job(dl, dsym)
    data, n = coder.to_bytes()
    for b in range(B):
        assert int(n[b]) == int(nb[b]) and data[b] == out[b, :(int(nb[b]) + 7) // 8].tobytes(), (i, b)
    coder.decode_open()
    assert torch.equal(coder.decode_logits(dl), dsym), (dtype, V, prec, B, steps, shape)
    coder.close()
