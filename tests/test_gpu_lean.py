"""The lean few-stream decode step (k_decode_lean, lac_decode.hip) and its hand-over to
k_decode_seq: streams that leave the lean case part-way -- a row whose total reaches
2^32, a fudged row (T > w*minp, arith_code.py:84) -- continue on k_decode_seq from the
step they stopped at, in the same launch chunk, and every path decodes the same symbols
as the one-launch wave kernel."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _roundtrip(pmf, sym, prec):
    from lac_amd.batch import BatchCoder
    T, B, V = pmf.shape
    c = BatchCoder(V, B, prec=prec, capacity_bits=T * (prec + 34) + 256, device=DEV)
    dp = torch.from_numpy(np.ascontiguousarray(pmf).view(np.int32)).to(DEV)
    c.encode_job(dp, torch.from_numpy(sym).to(DEV))
    c.raise_on_error()
    outs = {}
    for path in ("stats", "fused"):
        c.set_decode_path(path)
        c.decode_open()
        outs[path] = c.decode(dp).cpu().numpy()
    c.close()
    return outs


@pytest.mark.parametrize("prec", [24, 40, 50])
def test_lean_hands_over_mid_stream(prec):
    rng = np.random.default_rng(prec)
    V, B, T = 4000, 4, 300
    pmf = rng.integers(1, 1000, size=(T, B, V)).astype(np.uint32)
    pmf[120:, 0, :] = rng.integers(1 << 20, 1 << 21, size=(T - 120, V))   # totals > 2^32 from step 120
    pmf[77, 1, :] = 1 << 19                                             # T = 2^31 with minp 1:
    pmf[77, 1, 5] = 1                                                   # fudged at prec <= 31
    pmf[200:, 3, :] = rng.integers(1, 4, size=(T - 200, V))             # small totals
    sym = rng.integers(0, V, size=(T, B)).astype(np.int32)
    outs = _roundtrip(pmf, sym, prec)
    for path, o in outs.items():
        assert np.array_equal(o, sym), path


def test_lean_many_launch_chunks_and_ragged_vocab():
    """V = 32004 (a ragged last chunk and iteration) with enough streams that the lean
    buffers take 64 steps per launch: three launch chunks, the last partial."""
    from lac_amd import synth
    from lac_amd.batch import BatchCoder
    V, B, T, prec = 32004, 40, 140, 48
    pmf, sym = synth.softmax_tables(T, B, V, seed=77, device=DEV)
    c = BatchCoder(V, B, prec=prec, capacity_bits=T * (prec + 2) + 256, device=DEV)
    c.encode_job(pmf, sym)
    c.raise_on_error()
    for path in ("stats", "fused"):
        c.set_decode_path(path)
        c.decode_open()
        assert torch.equal(c.decode(pmf), sym), path
    c.close()


@pytest.mark.parametrize("mapping", ["floor", "ceil"])
def test_lean_mappings_agree_with_wave_path(mapping):
    """The floor mapping (Predictor / ACSampler ranges, no fudge) and the ceil mapping
    through the lean step give the wave kernel's symbols, at 1 and 5 streams (helpers on)."""
    from lac_amd.batch import BatchCoder
    rng = np.random.default_rng(11)
    for B in (1, 5):
        V, T, prec = 1000, 700, 36
        pmf = rng.integers(1, 5000, size=(T, B, V)).astype(np.uint32)
        sym = rng.integers(0, V, size=(T, B)).astype(np.int32)
        c = BatchCoder(V, B, prec=prec, capacity_bits=T * (prec + 16) + 256, device=DEV)
        c.set_mapping(mapping)
        dp = torch.from_numpy(pmf.view(np.int32)).to(DEV)
        c.encode_job(dp, torch.from_numpy(sym).to(DEV))
        c.raise_on_error()
        outs = []
        for path in ("stats", "fused"):
            c.set_decode_path(path)
            c.decode_open()
            outs.append(c.decode(dp).cpu().numpy())
        c.close()
        assert np.array_equal(outs[0], sym) and np.array_equal(outs[1], sym), (mapping, B)


def test_lean_total_at_2_32_boundary():
    """Rows with totals 2^32 - 1 (lean) and exactly 2^32 (k_decode_seq) interleaved in one
    stream; the vector CDF wraps mod 2^32 only on the rows the lean step refuses."""
    rng = np.random.default_rng(3)
    V, B, T, prec = 1024, 2, 200, 48
    base = np.full(V, (1 << 22), dtype=np.uint64)                # 1024 * 2^22 = 2^32
    pmf = np.empty((T, B, V), dtype=np.uint32)
    for t in range(T):
        for b in range(B):
            row = base.copy()
            if (t + b) % 3 == 0:
                row[rng.integers(V)] -= 1                            # 2^32 - 1: lean
            pmf[t, b] = row.astype(np.uint32)
    sym = rng.integers(0, V, size=(T, B)).astype(np.int32)
    outs = _roundtrip(pmf, sym, prec)
    for path, o in outs.items():
        assert np.array_equal(o, sym), path
