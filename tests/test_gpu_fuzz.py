"""Seeded random configurations through every encode and decode kernel.

Each case draws a vocabulary (odd sizes take the scalar-load kernels), a
precision, a row family (log-uniform, with zeros, peaked, flat, llama-scale
u64 rows that always take fudged_dist), a stream count and a step count, then
checks the GPU bytes of the split, fused and AUTO encoders against the C oracle
(oracle/lac_oracle.c, pinned to the reference's golden vectors) and decodes the
stream back with every decode kernel (per-step, one-wave fine and chunk, stats,
block).  Cases are fixed by the seed, so a failure reproduces exactly.
"""
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


@pytest.mark.parametrize("i", range(36))
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
