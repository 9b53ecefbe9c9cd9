"""Logits path on the GPU vs the C oracle.

The oracle side is ``oracle.q1_quantize`` (C restatement of the q1 quantiser,
itself checked against an independent numpy restatement in
tests/test_q1_quantiser.py) followed by ``oracle.encode_batch`` (the literal
restatement of CDFPredictor + A_to_bin, pinned to the reference's golden
vectors).  Everything is bit-exact: tables, bytes, lengths, traces, decodes.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _coder(V, B, prec, cap=None):
    from lac_amd.batch import BatchCoder
    return BatchCoder(V, B, prec=prec, pmf_bits=32, capacity_bits=cap, device=DEV)


def _logits(seed, steps, B, V, scale=3.0, specials=False):
    """Normal logits with a few sharp peaks (LLM-like), f32 host array."""
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((steps, B, V)) * scale).astype(np.float32)
    hot = rng.integers(0, V, size=(steps, B))
    np.put_along_axis(x, hot[..., None], np.float32(scale * 6), axis=2)
    if specials and V >= 16:
        x[0, 0, :3] = [np.nan, -np.inf, 1e30]
        if B > 1:
            x[0, 1, :] = -np.inf                                  # all -inf row: uniform table
        if steps > 1:
            x[1, 0, 5] = np.inf                                   # +inf max: every other entry 1
        if steps > 2:
            x[2, 0, 7] = 262143.5                                 # largest max of the GPU fast path
            x[2, 0, 9] = 262143.5 - 3.0
            x[2, B - 1, 3] = 3.0e5                                # just past it: capped (slow) path
            x[2, B - 1, 4] = 3.0e5 - 0.25
        if steps > 3 and B > 2:
            # row maxima the bf16 packed-int16 max must hand to the exact float path
            x[3, 0, :] = -np.abs(x[3, 0, :]) - 1.0                   # all negative
            x[3, 1, :] = -np.abs(x[3, 1, :]) - 1.0
            x[3, 1, 6] = -0.0                                     # max -0.0
            x[3, 2, :] = -np.abs(x[3, 2, :]) - 1.0
            x[3, 2, 11] = 0.0                                     # max +0.0, all else negative
            x[3, B - 1, 2] = np.float32(-np.nan)                  # negative NaN in a normal row
            x[1, B - 1, 8] = np.float32(np.nan)                   # positive NaN in a normal row
    return x


def _device_logits(x, dtype):
    t = torch.from_numpy(x).to(DEV)
    return t.to(torch.bfloat16) if dtype == "bf16" else t


def _host_bits(t):
    """The exact logits the GPU sees, for the oracle (bf16 as uint16 patterns)."""
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).cpu().numpy().view(np.uint16)
    return t.cpu().numpy()


def _sample(pmf, seed):
    """Symbols drawn from the tables themselves (inverse CDF), int32 [steps, B]."""
    rng = np.random.default_rng(seed)
    c = np.cumsum(pmf.astype(np.uint64), axis=-1)
    r = (rng.random(pmf.shape[:-1]) * c[..., -1]).astype(np.uint64)
    s = np.empty(pmf.shape[:-1], dtype=np.int32)
    for idx in np.ndindex(*pmf.shape[:-1]):
        s[idx] = np.searchsorted(c[idx], r[idx], side="right")
    return np.minimum(s, pmf.shape[-1] - 1).astype(np.int32)


CASES = [
    # V, B, steps, prec, dtype
    (32000, 64, 8, 48, "bf16"),
    (32000, 64, 8, 48, "f32"),
    (1000, 40, 30, 40, "f32"),
    (1000, 40, 30, 40, "bf16"),
    (128256, 8, 4, 48, "bf16"),            # 16-wave single-pass row stats
    (128256, 4, 5, 48, "f32"),             # rows split over a pair of blocks (shape 19)
    (131080, 6, 5, 48, "bf16"),            # bf16 row groups: the int16 max exchanged, float fallback rows
    (151936, 12, 4, 48, "bf16"),           # Qwen2: 5 row slots of 4-row blocks, fallback rows among them
    (65536, 6, 3, 48, "bf16"),             # (8,16) shape
    (24, 5, 50, 24, "f32"),
    (4096, 2048, 3, 48, "bf16"),
    (1000, 16, 20, 56, "bf16"),            # prec > 50: k_q1_decode's 128-bit division form
    (32000, 8, 6, 60, "f32"),
]


@pytest.mark.parametrize("V,B,steps,prec,dtype", CASES)
def test_logits_encode_decode_vs_oracle(V, B, steps, prec, dtype):
    from oracle import oracle as coracle
    x = _logits(V + B + prec, steps, B, V, specials=True)
    dl = _device_logits(x, dtype)
    c = _coder(V, B, prec, cap=steps * (prec + 2) + 256)
    # tables
    want_pmf = coracle.q1_quantize(_host_bits(dl), prec)
    got_pmf = c.quantize_logits(dl).cpu().numpy().view(np.uint32)
    assert (got_pmf == want_pmf).all()
    k = c.q1_k()
    assert want_pmf.max() <= 1 << k and want_pmf.min() >= 1
    # encode
    sym = _sample(want_pmf, V + 1)
    trace = torch.zeros((steps, B, 2), dtype=torch.int64, device=DEV)
    c.encode_logits_job(dl, torch.from_numpy(sym).to(DEV), trace=trace)
    data, n = c.to_bytes()
    out, nb, status, rc = coracle.encode_batch(want_pmf, sym, prec, nthreads=16)
    assert rc == 0 and not status.any()
    for b in range(B):
        assert int(n[b]) == int(nb[b]), b
        assert data[b] == out[b, :(int(nb[b]) + 7) // 8].tobytes(), b
    # the same tables through the pmf path give the same trace and bits
    c2 = _coder(V, B, prec, cap=steps * (prec + 2) + 256)
    trace2 = torch.zeros_like(trace)
    c2.encode_job(torch.from_numpy(want_pmf.view(np.int32)).to(DEV), torch.from_numpy(sym).to(DEV), trace=trace2)
    assert torch.equal(trace, trace2)
    # decode from logits (own bits), and from the oracle's bits
    c.decode_open()
    dec = c.decode_logits(dl).cpu().numpy()
    assert (dec == sym).all()
    stride = (out.shape[1] + 7) // 8 * 8
    buf = np.zeros((B, stride), dtype=np.uint8)
    buf[:, :out.shape[1]] = out
    c.decode_open(torch.from_numpy(buf).to(DEV), torch.from_numpy(nb.astype(np.int64)).to(DEV))
    assert (c.decode_logits(dl).cpu().numpy() == sym).all()
    assert (c.determined() <= steps).all()
    c.raise_on_error()


def test_logits_headline_shape_matches_pmf_path():
    """Full c3 shape (V=32000, B=4096): fused logits kernel == quantise + pmf kernel."""
    V, B, steps, prec = 32000, 4096, 3, 48
    g = torch.Generator(device=DEV).manual_seed(3)
    dl = (torch.randn((steps, B, V), device=DEV, generator=g) * 3).to(torch.bfloat16)
    c = _coder(V, B, prec)
    pmf = c.quantize_logits(dl)
    sym = torch.randint(0, V, (steps, B), device=DEV, generator=g, dtype=torch.int32)
    c.encode_logits_job(dl, sym)
    a, na = c.to_bytes()
    c2 = _coder(V, B, prec)
    c2.encode_job(pmf, sym)
    b, nb = c2.to_bytes()
    assert (na == nb).all() and a == b
    c.decode_open()
    assert torch.equal(c.decode_logits(dl), sym)


def test_logits_broadcast_and_strides():
    """A stride-0 step broadcast and a padded stream stride give the same bits."""
    from oracle import oracle as coracle
    V, B, steps, prec = 512, 16, 12, 40
    x = _logits(9, 1, B, V)
    pad = torch.zeros((B, V + 64), dtype=torch.float32, device=DEV)
    pad[:, :V] = torch.from_numpy(x[0]).to(DEV)
    row = pad[:, :V].unsqueeze(0).expand(steps, B, V)              # step stride 0, stream stride V+64
    want = coracle.q1_quantize(x[0], prec)
    sym = np.stack([_sample(want, s) for s in range(steps)])
    c = _coder(V, B, prec)
    c.encode_logits_job(row, torch.from_numpy(sym).to(DEV))
    data, n = c.to_bytes()
    out, nb, _, rc = coracle.encode_batch(np.broadcast_to(want, (steps, B, V)).copy(), sym, prec, nthreads=8)
    assert rc == 0
    assert [out[b, :(int(nb[b]) + 7) // 8].tobytes() for b in range(B)] == data
    c.decode_open()
    assert (c.decode_logits(row).cpu().numpy() == sym).all()


def test_logits_errors():
    from lac_amd._lib import LacError, LAC_E_ARG, LAC_E_STATE, LAC_E_PREC, LAC_E_SYMBOL_RANGE
    from lac_amd.batch import StreamError
    c = _coder(1004, 4, 40)                                        # 1004 % 8 != 0
    bf = torch.zeros((2, 4, 1004), dtype=torch.bfloat16, device=DEV)
    with pytest.raises(LacError) as e:
        c.encode_logits_job(bf, torch.zeros((2, 4), dtype=torch.int32, device=DEV))
    assert e.value.code == LAC_E_ARG
    f = torch.zeros((2, 4, 1004), dtype=torch.float32, device=DEV)  # f32 needs V % 4 == 0: fine
    c.encode_logits_job(f, torch.tensor([[0, 1, 2, 1003], [5, 6, 7, 8]], dtype=torch.int32, device=DEV))
    c.raise_on_error()
    c.set_mapping("floor")
    with pytest.raises(LacError) as e:
        c.encode_logits_job(f, torch.zeros((2, 4), dtype=torch.int32, device=DEV))
    assert e.value.code == LAC_E_STATE
    c.set_mapping("ceil")
    c.encode_logits_job(f, torch.tensor([[0, 1, 1004, 1], [5, -1, 7, 8]], dtype=torch.int32, device=DEV))
    with pytest.raises(StreamError) as e:
        c.raise_on_error()
    assert e.value.code == LAC_E_SYMBOL_RANGE
    assert list(e.value.err != 0) == [False, True, True, False]
    tight = _coder(1 << 20, 1, 22)                                 # prec-1-ceil(log2 V) = 1: ok
    assert tight.q1_k() == 1
    with pytest.raises(LacError) as e:
        _coder(1 << 20, 1, 21).quantize_logits(torch.zeros((1, 1, 1 << 20), device=DEV))
    assert e.value.code == LAC_E_PREC


def test_logits_decode_spans_step_chunks():
    """600 streams x 70 steps of logits: both q1 kernels run in 64-step chunks."""
    V, B, steps, prec = 1024, 600, 70, 40
    g = torch.Generator(device=DEV).manual_seed(4)
    dl = (torch.randn((steps, B, V), device=DEV, generator=g) * 4).to(torch.bfloat16)
    c = _coder(V, B, prec, cap=steps * (prec + 2) + 256)
    sym = torch.randint(0, V, (steps, B), device=DEV, generator=g, dtype=torch.int32)
    c.encode_logits_job(dl, sym)
    a, na = c.to_bytes()
    c2 = _coder(V, B, prec, cap=steps * (prec + 2) + 256)
    c2.encode_job(c.quantize_logits(dl), sym)
    assert c2.to_bytes()[0] == a
    c.decode_open()
    assert torch.equal(c.decode_logits(dl), sym)


def test_incremental_logits_encode_mixes_with_pmf_steps():
    """encode_logits (no reset/finish) in pieces, interleaved with pmf steps of the
    same q1 tables, equals one encode_logits_job."""
    V, B, steps, prec = 1024, 48, 40, 40
    g = torch.Generator(device=DEV).manual_seed(6)
    dl = (torch.randn((steps, B, V), device=DEV, generator=g) * 3).to(torch.bfloat16)
    sym = torch.randint(0, V, (steps, B), device=DEV, generator=g, dtype=torch.int32)
    c = _coder(V, B, prec, cap=steps * (prec + 2) + 256)
    c.encode_logits_job(dl, sym)
    one, n1 = c.to_bytes()
    pmf = c.quantize_logits(dl)
    c2 = _coder(V, B, prec, cap=steps * (prec + 2) + 256)
    c2.reset()
    for a, b, kind in ((0, 7, "logits"), (7, 8, "pmf"), (8, 30, "logits"), (30, 40, "pmf")):
        if kind == "logits":
            c2.encode_logits(dl[a:b], sym[a:b].contiguous())
        else:
            c2.encode(pmf[a:b], sym[a:b].contiguous())
    c2.finish()
    two, n2 = c2.to_bytes()
    assert (n1 == n2).all() and one == two


@pytest.mark.parametrize("dtype,V", [("bf16", 32000), ("f32", 32000), ("bf16", 128256), ("f32", 65536),
                                     ("bf16", 128512), ("bf16", 128520), ("f32", 65540), ("f32", 128256),
                                     ("f32", 128512), ("f32", 128520), ("bf16", 131080), ("bf16", 151936),
                                     ("f32", 151936), ("bf16", 262144), ("f32", 256000), ("f32", 262144),
                                     ("bf16", 163840), ("bf16", 163848), ("f32", 81920), ("f32", 81924),
                                     ("bf16", 202048), ("bf16", 208896), ("bf16", 208904), ("f32", 102400)])
def test_every_q1_shape_gives_the_same_bits(dtype, V):
    """Every forced row-stats shape (8/16-wave blocks, tiles, rolling prefetch,
    registers + LDS slots) yields the AUTO shape's bytes and decodes; shapes that
    cannot hold the row are refused with LAC_E_ARG.  V = 128256 bf16 and 65536
    f32 fill the register + LDS shape (15) exactly up to its 16384 vectors; bf16
    128512 / 128520 sit on either side of its 16-copy form's 16064-vector limit.
    Rows past 16384 vectors take row groups (19 / 20 / 21: segments in row slots
    of 1 / 2 / 4 rows per block; forced, they also split shorter rows): 2 slots at
    f32 65540 .. 128520 in the 1-row form, 5 slots of the 4-row form at bf16
    131080 / 151936 and f32 65540, 5 of the 2-row form at f32 151936, 9 at bf16
    262144, 2 / 4 of the 8-copy 1-row form at f32 256000 / 262144 (Gemma 3).
    Rows of 16385..20480 vectors take one 8-wave block each, in registers (22: bf16
    131080 / 151936 / 163840, f32 65540 / 81920), up to 26112 with 11 more vectors
    per thread in LDS slots (22: bf16 163848 / 202048 / 208896, f32 81924 /
    102400); longer ones where the slot form would put several rows in a block and
    the blocks fill well take groups of such blocks (23: bf16 262144, f32 151936);
    forced, 23 also splits shorter rows."""
    from lac_amd._lib import LacError
    B, steps, prec = 12, 3, 48
    x = _logits(777, steps, B, V, specials=True)
    dl = _device_logits(x, dtype)
    c = _coder(V, B, prec, cap=steps * (prec + 2) + 256)
    pmf = c.quantize_logits(dl).cpu().numpy().view(np.uint32)
    sym = torch.from_numpy(_sample(pmf, 5)).to(DEV)
    c.encode_logits_job(dl, sym)
    want, wn = c.to_bytes()
    ran = 0
    for sh in range(1, 24):
        try:
            c.set_q1_shape(sh)                # retired shapes are refused here
            c.encode_logits_job(dl, sym)      # and shapes that cannot hold the row here
        except LacError:
            continue
        got, gn = c.to_bytes()
        assert got == want and (gn == wn).all(), sh
        c.decode_open()
        assert torch.equal(c.decode_logits(dl), sym), sh
        ran += 1
    assert ran >= (6 if V == 32000 else 3)
    c.close()


@pytest.mark.parametrize("dtype,V,B,steps", [("f32", 65540, 300, 70), ("f32", 128256, 520, 3),
                                             ("bf16", 256000, 300, 3), ("bf16", 262144, 64, 3),
                                             ("f32", 151936, 256, 3), ("f32", 262144, 128, 3),
                                             ("bf16", 151936, 300, 3), ("bf16", 131080, 333, 3)])
def test_paired_row_stats_many_rows(dtype, V, B, steps):
    """Rows split into row groups with many rounds per launch and, at 70 steps, two
    launches per job (the sequence numbers and maximum words are cleared): logits
    path bytes == quantise + pmf path, decode round trip, and == the tiled shape's
    and every forced group form's bytes (rounds with a partial last one: 333 x 3
    rows over 25 rows per XCD per round)."""
    g = torch.Generator(device=DEV).manual_seed(V + B)
    dl = torch.randn((steps, B, V), device=DEV, generator=g) * 3
    if dtype == "bf16":
        dl = dl.to(torch.bfloat16)
    prec = 48
    c = _coder(V, B, prec, cap=steps * (prec + 2) + 256)
    sym = torch.randint(0, V, (steps, B), device=DEV, generator=g, dtype=torch.int32)
    c.encode_logits_job(dl, sym)
    a, na = c.to_bytes()
    for sh in (14, 19, 20, 21, 23) + ((22,) if V // (8 if dtype == "bf16" else 4) <= 26112 else ()):
        c.set_q1_shape(sh)
        c.encode_logits_job(dl, sym)
        assert c.to_bytes()[0] == a, sh
    c.set_q1_shape(0)
    pmf = c.quantize_logits(dl)
    c2 = _coder(V, B, prec, cap=steps * (prec + 2) + 256)
    c2.encode_job(pmf, sym)
    b, nb = c2.to_bytes()
    assert (na == nb).all() and a == b
    del pmf, c2
    c.decode_open()
    assert torch.equal(c.decode_logits(dl), sym)
    c.raise_on_error()


def test_q1_shape_option_range():
    """LAC_OPT_Q1_SHAPE takes 0 (AUTO) and the live shapes of 1 .. 23; anything else,
    the retired shapes included (5, 7, 9, 11, 12, 13, 16: AUTO never took them), is
    refused with LAC_E_ARG."""
    from lac_amd._lib import LacError, LAC_E_ARG
    c = _coder(1024, 4, 40)
    for bad in (-1, 5, 7, 9, 11, 12, 13, 16, 24, 99, 1 << 32 | 1):
        with pytest.raises(LacError) as e:
            c.set_q1_shape(bad)
        assert e.value.code == LAC_E_ARG
    for ok in (0, 1, 2, 3, 4, 6, 8, 10, 14, 15, 17, 18, 19, 20, 21, 22, 23):
        c.set_q1_shape(ok)
    c.close()


@pytest.mark.parametrize("hog_s,shape", [(0.6, 0), (0.02, 0), (0.6, 23)])
def test_row_groups_while_another_kernel_holds_cus(hog_s, shape):
    """Rows over groups of blocks (f32 V = 128256: shape 19, AUTO; or forced 23,
    groups of 8-wave blocks) need every group
    member resident.  A kernel on another stream holds all but 8 CUs (tests/native/
    hog.hip): for 0.6 s the waiting members give up, the launch aborts and the
    gated tiled launch recomputes every row; for 0.02 s the late members arrive in
    time.  The hog leaves one CU per XCD free, so the first block of each XCD's
    first group is resident and its partner is not.  Either way encode bytes and
    decoded symbols equal a run on an idle GPU."""
    import ctypes as C
    import os
    import time
    from conftest import REPO
    from lac_amd import _lib
    hog = C.CDLL(os.path.join(REPO, "tests", "native", "libhog.so"))
    hog.hog_launch.argtypes = [C.c_int, C.c_double, C.c_void_p, C.c_void_p]
    V, B, steps, prec = 128256, 256, 2, 48
    x = _device_logits(_logits(31, steps, B, V), "f32")
    c = _coder(V, B, prec, cap=steps * (prec + 2) + 256)
    q = c.quantize_logits(x)
    cdf = torch.cumsum(q.view(torch.int32).to(torch.int64) & 0xFFFFFFFF, -1)
    u = torch.rand((steps, B, 1), generator=torch.Generator(device=DEV).manual_seed(5), device=DEV,
                   dtype=torch.float64)
    sym = torch.searchsorted(cdf, (u * cdf[..., -1:].double()).long(), right=True).squeeze(-1).to(torch.int32)
    sym = torch.clamp(sym, max=V - 1)
    c.encode_logits_job(x, sym)
    want, wn = c.to_bytes()
    c.set_q1_shape(shape)
    ok = torch.zeros(1, dtype=torch.int32, device=DEV)
    busy = torch.cuda.Stream(device=DEV)
    mine = torch.cuda.Stream(device=DEV)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    assert hog.hog_launch(1, 0.001, C.c_void_p(ok.data_ptr()), C.c_void_p(busy.cuda_stream)) == 0   # code loaded
    torch.cuda.synchronize()
    ok.zero_()
    assert hog.hog_launch(cus - 8, hog_s, C.c_void_p(ok.data_ptr()), C.c_void_p(busy.cuda_stream)) == 0
    time.sleep(min(0.1, hog_s / 4))                               # the hog holds its CUs before we launch
    t_enc = time.perf_counter()
    with torch.cuda.stream(mine):
        c.encode_logits_job(x, sym)
        mine.synchronize()
        t_enc = time.perf_counter() - t_enc
        aborted_enc = C.c_int64()
        _lib.check(c.lib.lac_q1_group_aborted(c.ctx, C.byref(aborted_enc), c._stream))
        got, gn = c.to_bytes()
    torch.cuda.synchronize()
    assert got == want and (gn == wn).all()
    assert hog.hog_launch(cus - 8, hog_s, C.c_void_p(ok.data_ptr()), C.c_void_p(busy.cuda_stream)) == 0
    time.sleep(min(0.1, hog_s / 4))
    t_dec = time.perf_counter()
    with torch.cuda.stream(mine):
        c.decode_open()
        dec = c.decode_logits(x)
        mine.synchronize()
        t_dec = time.perf_counter() - t_dec
        aborted_dec = C.c_int64()
        _lib.check(c.lib.lac_q1_group_aborted(c.ctx, C.byref(aborted_dec), c._stream))
        c.raise_on_error()
    torch.cuda.synchronize()
    assert torch.equal(dec, sym)
    assert int(ok.item()) == 2 * (cus - 8)                        # both hogs ran to their deadline
    if hog_s > 0.3:
        # the abort path was taken (which launch meets the missing partner first depends
        # on how the dispatcher fills the free CUs: tools/contention_probe.py saw both)
        assert aborted_enc.value or aborted_dec.value, (t_enc, t_dec)
    c.close()
