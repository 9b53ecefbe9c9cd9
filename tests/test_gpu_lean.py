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


# ---- round 6: u64 tables (totals below 2^50), static rows, LAC_OPT_DECODE_STOP

def _dev(a):
    a = np.ascontiguousarray(a)
    return torch.from_numpy(a.view(np.int32) if a.dtype == np.uint32 else a.view(np.int64)).to(DEV)


def _oracle_bits(pmf, sym, prec):
    """The C oracle's bitstreams (test infrastructure) -> device bits [B, stride], nbits."""
    from oracle import oracle as coracle
    out, onb, _, rc = coracle.encode_batch(pmf, sym, prec)
    assert rc == 0
    B = pmf.shape[1]
    stride = ((out.shape[1] + 7) // 8 + 1) * 8
    buf = np.zeros((B, stride), dtype=np.uint8)
    buf[:, :out.shape[1]] = out
    return torch.from_numpy(buf).to(DEV), torch.from_numpy(onb.astype(np.int64)).to(DEV)


@pytest.mark.parametrize("prec", [40, 50, 51])
def test_lean_u64_totals_between_2_32_and_2_50(prec):
    """u64 tables with totals in (2^32, 2^50): the lean step (prec <= 50) decodes the C
    oracle's bitstreams to the encoded symbols, as the wave kernel does; rows at 2^50 - 1
    (lean) and 2^50 (k_decode_seq) interleave, and a fudged row (T > w * minp) hands over
    mid-stream.  prec 51 takes k_decode_seq throughout."""
    from lac_amd.batch import BatchCoder
    rng = np.random.default_rng(prec)
    V, B, T = 3000, 3, 260
    pmf = rng.integers(1 << 20, 1 << 24, size=(T, B, V)).astype(np.uint64)   # totals ~2^35
    pmf[:, 1, :] = rng.integers(1 << 30, 1 << 36, size=(T, V))               # totals ~2^47
    for t in range(0, T, 7):                                                 # 2^50 - 1 / 2^50 rows
        row = np.full(V, (1 << 50) // V, dtype=np.uint64)
        row[0] += (1 << 50) - int(row.sum()) - (t % 2)
        pmf[t, 2] = row
    pmf[90, 0, :] = 1 << 37                                                  # T ~ 2^48.6, minp 1:
    pmf[90, 0, 11] = 1                                                       # fudged below prec 50
    sym = rng.integers(0, V, size=(T, B)).astype(np.int32)
    bits, nbits = _oracle_bits(pmf, sym, prec)
    c = BatchCoder(V, B, prec=prec, pmf_bits=64, capacity_bits=T * (prec + 2) + 256, device=DEV)
    dp = _dev(pmf)
    for path in ("stats", "fused"):
        c.set_decode_path(path)
        c.decode_open(bits, nbits)
        assert np.array_equal(c.decode(dp).cpu().numpy(), sym), path
    c.close()


@pytest.mark.parametrize("bits_", [32, 64])
@pytest.mark.parametrize("prec", [24, 48])
def test_static_rows_one_stats_row_per_stream(bits_, prec):
    """A static model (stride-0 steps) takes its row statistics once per stream: 3000 steps
    in one launch pair, the stats path equal to the wave path; at prec 24 the row fudges
    (T > w * minp) on some steps, which k_decode_seq takes with the same one row."""
    from lac_amd.batch import BatchCoder
    rng = np.random.default_rng(bits_ + prec)
    V, B, T = 2000, 2, 3000
    dt = np.uint32 if bits_ == 32 else np.uint64
    row = rng.integers(1, 1 << 14, size=(B, V)).astype(dt)
    row[1, 7] = 1                                                            # minp 1
    sym = rng.integers(0, V, size=(T, B)).astype(np.int32)
    pmf = np.broadcast_to(row[None], (T, B, V))
    c = BatchCoder(V, B, prec=prec, pmf_bits=bits_, capacity_bits=T * (prec + 2) + 256, device=DEV)
    dp = _dev(row).view(1, B, V).expand(T, B, V)
    c.encode_job(dp, torch.from_numpy(sym).to(DEV))
    c.raise_on_error()
    data, nb = c.to_bytes()
    from oracle import oracle as coracle
    out, onb, _, rc = coracle.encode_batch(np.ascontiguousarray(pmf), sym, prec)
    for b in range(B):
        assert int(nb[b]) == int(onb[b]) and data[b] == out[b, :(int(onb[b]) + 7) // 8].tobytes()
    for path in ("stats", "fused"):
        c.set_decode_path(path)
        c.decode_open()
        assert np.array_equal(c.decode(dp).cpu().numpy(), sym), path
    c.close()


@pytest.mark.parametrize("storage", [32, 64])
def test_decode_stop_at_reference_count(storage):
    """LAC_OPT_DECODE_STOP: decoding past a stream's end, each stream stops by itself
    before the first symbol its bits do not determine -- after exactly the symbols the
    reference's bit-serial run(bits, stop=0) emits (decoded_count of the reference-run
    fixtures: the encoded symbols and the extra ones, rows past the end repeating the last,
    as the fixtures' Replay predictor) -- with LAC_E_UNDETERMINED, the lean step (prec <= 50)
    and k_decode_seq alike."""
    from conftest import load_golden
    from lac_amd import synth
    from lac_amd.batch import BatchCoder
    from lac_amd import _lib
    from lac_amd.coder import _DEC_STATE
    import ctypes as C
    cases = [c for c in load_golden("gen_cases.json") + load_golden("straight_cases.json") if "decoded_count" in c]
    assert len(cases) >= 10
    for case in cases:
        rows = np.stack([synth.pmf_row(case["seed"], t, 0, case["V"], case["kind"], case["exp_range"])
                         for t in range(case["steps"])])
        if storage == 32 and rows.dtype != np.uint32:
            continue
        rows = rows.astype(np.uint32 if storage == 32 else np.uint64)
        T, V, prec, n = case["steps"], case["V"], case["prec"], case["decoded_count"]
        extra = n - T + 20
        pmf = np.concatenate([rows, np.repeat(rows[-1:], extra, axis=0)])[:, None, :]
        L = case["L"]
        data = bytes.fromhex(case["bytes"])
        buf = np.zeros((1, ((len(data) + 7) // 8 + 1) * 8), dtype=np.uint8)
        buf[0, :len(data)] = np.frombuffer(data, dtype=np.uint8)
        c = BatchCoder(V, 1, prec=prec, pmf_bits=storage, capacity_bits=64, device=DEV)
        c.set_decode_stop(True)
        c.decode_open(torch.from_numpy(buf).to(DEV), torch.tensor([L], dtype=torch.int64, device=DEV))
        out = c.decode(_dev(pmf)).cpu().numpy()[:, 0]
        st = np.zeros(1, dtype=_DEC_STATE)
        _lib.check(c.lib.lac_decode_get_state(c.ctx, st.ctypes.data_as(C.c_void_p), c._stream))
        want = case["syms"] + case["decoded_extra"]
        assert int(st["err"][0]) == _lib.LAC_E_UNDETERMINED and int(st["err_step"][0]) == n, (case["name"], st)
        assert int(st["nsym"][0]) == n and int(st["ndet"][0]) == n, case["name"]
        assert out[:n].tolist() == want and (out[n:] == -1).all(), case["name"]
        c.close()


@pytest.mark.parametrize("prec", [30, 48, 50])
def test_lean_u64_wide_totals(prec):
    """u64 rows with totals of 2^50 and more take the lean step's wide form (the search
    against a double window around the target, the ranges by div_mid): llama-scale tables (max(2,
    floor(softmax * 2^60)), bench --pmf-bits 64), rows with totals in [2^63, 2^64) and
    just below 2^64, all against the C oracle's bitstreams and the wave kernel."""
    from lac_amd import synth
    from lac_amd.batch import BatchCoder
    V, B, T = 4000, 3, 300
    pmf_d, sym_d = synth.softmax_tables(T, B, V, seed=5 + prec, device=DEV, scale_bits=60, storage_bits=64)
    pmf = pmf_d.cpu().numpy().view(np.uint64).copy()
    sym = sym_d.cpu().numpy()
    rng = np.random.default_rng(prec)
    for t in range(0, T, 5):                                    # stream 2: totals in [2^63, 2^64)
        row = rng.integers(1 << 40, 1 << 51, size=V).astype(np.uint64)
        row = (row.astype(object) * ((1 << 63) + int(rng.integers(0, 1 << 62))) // int(row.sum())).astype(np.uint64)
        row[0] += np.uint64(t % 3)
        pmf[t, 2] = np.maximum(row, 1)
    pmf[7, 1, :] = np.uint64(((1 << 64) - 1) // V)             # just below 2^64
    pmf[7, 1, 0] += np.uint64(((1 << 64) - 1) % V)
    assert int(pmf[7, 1].astype(object).sum()) == (1 << 64) - 1
    bits, nbits = _oracle_bits(pmf, sym, prec)
    c = BatchCoder(V, B, prec=prec, pmf_bits=64, capacity_bits=T * (prec + 2) + 256, device=DEV)
    dp = _dev(pmf)
    for path in ("stats", "fused"):
        c.set_decode_path(path)
        c.decode_open(bits, nbits)
        assert np.array_equal(c.decode(dp).cpu().numpy(), sym), path
    c.close()


def test_lean_many_groups_two_streams():
    """V = 32000 u32 with 2 streams: the 512 MB lean buffers hold 2048 steps' rows, so
    4000 steps are two launch groups; one stream leaves the lean case (totals >= 2^32)
    for 100 steps inside the first group and comes back in it."""
    from lac_amd.batch import BatchCoder
    rng = np.random.default_rng(21)
    V, B, T, prec = 32000, 2, 4000, 48
    pmf = rng.integers(1, 60000, size=(T, B, V)).astype(np.uint32)
    pmf[1500:1600, 1, :] = rng.integers(1 << 17, 1 << 18, size=(100, V))   # totals > 2^32
    sym = rng.integers(0, V, size=(T, B)).astype(np.int32)
    c = BatchCoder(V, B, prec=prec, capacity_bits=T * (prec + 20) + 256, device=DEV)
    dp = torch.from_numpy(pmf.view(np.int32)).to(DEV)
    c.encode_job(dp, torch.from_numpy(sym).to(DEV))
    c.raise_on_error()
    for path in ("stats", "fused"):
        c.set_decode_path(path)
        c.decode_open()
        got = c.decode(dp).cpu().numpy()
        assert np.array_equal(got, sym), (path, np.argwhere(got != sym)[:4])
    c.close()


@pytest.mark.parametrize("prec", [49, 50])
def test_lean_u64_wide_clustered_entries(prec):
    """Wide rows (totals near 2^60) whose small entries (4096 .. 8191, so the ceil mapping
    is never fudged at prec >= 49) sit closer together than the search's double window:
    targets among them make the window ambiguous and the search reruns with products.
    Most symbols are drawn from that cluster; against the C oracle and the wave kernel."""
    from lac_amd.batch import BatchCoder
    rng = np.random.default_rng(prec)
    V, B, T = 2000, 2, 300
    pmf = rng.integers(4096, 8192, size=(T, B, V)).astype(np.uint64)
    big = rng.choice(V, size=(T, B, 8))
    for t in range(T):
        for b in range(B):
            pmf[t, b, big[t, b]] = rng.integers(1 << 56, 1 << 57, size=8).astype(np.uint64)
    sym = rng.integers(0, V, size=(T, B)).astype(np.int32)
    pick_big = rng.random((T, B)) < 0.2
    for t in range(T):
        for b in range(B):
            if pick_big[t, b]:
                sym[t, b] = big[t, b, rng.integers(0, 8)]
    bits, nbits = _oracle_bits(pmf, sym, prec)
    c = BatchCoder(V, B, prec=prec, pmf_bits=64, capacity_bits=T * (prec + 2) + 256, device=DEV)
    dp = _dev(pmf)
    for path in ("stats", "fused"):
        c.set_decode_path(path)
        c.decode_open(bits, nbits)
        assert np.array_equal(c.decode(dp).cpu().numpy(), sym), path
    c.close()


@pytest.mark.parametrize("V", [20000, 65536])
def test_lean_u64_two_chunk_bounds_per_lane(V):
    """u64 rows carry up to 128 chunk bounds, two per lane (lean_chunk_layout): V = 20000
    puts chunks 64.. in the lanes' second bound, V = 65536 (four iterations per chunk) is
    the widest u64 row the lean step takes.  Llama-scale tables against the C oracle's
    bitstreams and the wave kernel."""
    from lac_amd import synth
    from lac_amd.batch import BatchCoder
    B, T, prec = 2, 200, 48
    pmf_d, sym_d = synth.softmax_tables(T, B, V, seed=V, device=DEV, scale_bits=60, storage_bits=64)
    pmf = pmf_d.cpu().numpy().view(np.uint64).copy()
    sym = sym_d.cpu().numpy()
    bits, nbits = _oracle_bits(pmf, sym, prec)
    c = BatchCoder(V, B, prec=prec, pmf_bits=64, capacity_bits=T * (prec + 2) + 256, device=DEV)
    dp = _dev(pmf)
    for path in ("stats", "fused"):
        c.set_decode_path(path)
        c.decode_open(bits, nbits)
        assert np.array_equal(c.decode(dp).cpu().numpy(), sym), path
    c.close()
