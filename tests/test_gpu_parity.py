"""GPU parity: liblac.so (HIP, gfx950) vs the oracle and the reference's golden vectors.

Every test calls the product through its C-ABI (lac_amd.batch -> liblac.so).
Integer/byte work, so the bar is bit-exact everywhere.
"""
import hashlib

import numpy as np
import pytest

from conftest import load_golden
from lac_amd import synth

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _coder(V, B, prec, bits=32, cap=1 << 16):
    from lac_amd.batch import BatchCoder
    return BatchCoder(V, B, prec=prec, pmf_bits=bits, capacity_bits=cap, device=DEV)


def _dev_pmf(a):
    """numpy uint32/uint64 -> int32/int64 device tensor with the same bits."""
    a = np.ascontiguousarray(a)
    view = a.view(np.int32) if a.dtype == np.uint32 else a.view(np.int64)
    return torch.from_numpy(view).to(DEV)


def _gpu_encode(pmf_np, sym_np, prec, trace=False, path="auto", job=False):
    steps, B, V = pmf_np.shape
    bits = 64 if pmf_np.dtype == np.uint64 else 32
    c = _coder(V, B, prec, bits, cap=steps * (prec + 2) + 256)
    c.set_path(path)
    pmf = _dev_pmf(pmf_np)
    sym = torch.from_numpy(np.ascontiguousarray(sym_np, dtype=np.int32)).to(DEV)
    tr = torch.zeros((steps, B, 2), dtype=torch.int64, device=DEV) if trace else None
    if job:
        c.encode_job(pmf, sym, trace=tr)
    else:
        c.encode(pmf, sym, trace=tr)
        c.finish()
    data, n = c.to_bytes()
    return c, pmf, data, n, tr


DECODE_PATHS = ("split", "fused", "fused_chunk", "stats", "block")


def _decode_both(c, dpmf):
    """Decode with the per-step workgroup kernel, the one-launch wave kernel and
    the stats path; all must agree.  Returns the symbols."""
    outs = []
    for path in DECODE_PATHS:
        c.set_decode_path(path)
        c.decode_open()
        outs.append(c.decode(dpmf).cpu().numpy())
    c.set_decode_path("auto")
    for o in outs[1:]:
        assert (outs[0] == o).all()
    return outs[0]


def _digits_from_trace(tr, b):
    from lac_amd.batch import digits_of
    t = tr[:, b, :].cpu().numpy()
    return [digits_of(int(E), int(k)) for E, k in t]


# ---------------------------------------------------------------- golden vectors
@pytest.mark.parametrize("path", ["split", "fused"])
@pytest.mark.parametrize("case", load_golden("gen_cases.json"), ids=lambda c: c["name"])
def test_golden_gen_case(case, path):
    rows = np.stack([synth.pmf_row(case["seed"], t, 0, case["V"], case["kind"], case["exp_range"])
                     for t in range(case["steps"])])
    pmf = rows[:, None, :]
    sym = np.asarray(case["syms"], dtype=np.int32)[:, None]
    c, dpmf, data, n, tr = _gpu_encode(pmf, sym, case["prec"], trace=True, path=path)
    assert int(n[0]) == case["L"] and data[0].hex() == case["bytes"]
    assert _digits_from_trace(tr, 0) == case["trace"]
    assert c.flush_digits()[0] == case["flush"]
    out = _decode_both(c, dpmf)[:, 0]
    assert out.tolist() == case["syms"]
    c.raise_on_error()


@pytest.mark.parametrize("path", ["split", "fused"])
def test_golden_small_cases(path):
    for kind in ("static", "perstep"):
        for c in load_golden("small_cases.json")[kind]:
            if not c["syms"]:
                continue
            T = len(c["syms"])
            rows = np.array(c["rows"], dtype=np.uint32)
            rows = rows if rows.shape[0] == T else np.repeat(rows[:1], T, axis=0)
            cd, dpmf, data, n, tr = _gpu_encode(rows[:, None, :], np.array(c["syms"])[:, None], c["prec"], trace=True,
                                                path=path)
            assert int(n[0]) == c["L"] and data[0].hex() == c["bytes"], c
            assert _digits_from_trace(tr, 0) == c["trace"]
            assert cd.flush_digits()[0] == c["flush"]
            assert _decode_both(cd, dpmf)[:, 0].tolist() == c["syms"]
            cd.close()


STRAIGHT_FIX = load_golden("straight_cases.json")


def _storages(rows):
    """The fixture's rows in u32 (where they fit) and u64 storage: the reference's output
    does not depend on it, and each storage reaches other straight encode forms."""
    out = [rows.astype(np.uint64)]
    if rows.dtype == np.uint32:
        out.insert(0, rows)
    return out


@pytest.mark.parametrize("case", load_golden("gen_cases.json") + STRAIGHT_FIX, ids=lambda c: c["name"])
def test_golden_untraced_straight(case):
    """Untraced split-path encodes -- the only ones that take k_encode's straight 64-step
    blocks (lac_encode.hip; a trace buffer sends every block to the general loop) -- of
    the reference-run fixtures, in u32 and u64 storage, and the untraced fused job: bytes
    and bit counts equal the reference's.  tests/straight_forms.py predicts which form
    each block takes; test_oracle_golden.py checks that these fixtures reach all of them
    (u32; u64 t32 / t32+ft / wide / wide+ft and both fudge exits)."""
    from straight_forms import forms_reached
    rows = np.stack([synth.pmf_row(case["seed"], t, 0, case["V"], case["kind"], case["exp_range"])
                     for t in range(case["steps"])])
    sym = np.asarray(case["syms"], dtype=np.int32)[:, None]
    for r in _storages(rows):
        for path, job in (("split", False), ("split", True), ("fused", True)):
            c, dpmf, data, n, _ = _gpu_encode(r[:, None, :], sym, case["prec"], path=path, job=job)
            assert int(n[0]) == case["L"] and data[0].hex() == case["bytes"], (r.dtype, path, job,
                                                                                forms_reached(r, case["syms"], case["prec"], r.dtype.itemsize * 8))
            c.close()


def test_golden_small_cases_untraced_straight():
    """The 500 small reference cases, untraced on the split path, u32 and u64 storage
    (the u32 form and the u64 t32 / t32+ft forms with the fudge exit, tests/straight_forms.py)."""
    for kind in ("static", "perstep"):
        for c in load_golden("small_cases.json")[kind]:
            if not c["syms"]:
                continue
            T = len(c["syms"])
            rows = np.array(c["rows"], dtype=np.uint32)
            rows = rows if rows.shape[0] == T else np.repeat(rows[:1], T, axis=0)
            for r in _storages(rows):
                cd, dpmf, data, n, _ = _gpu_encode(r[:, None, :], np.array(c["syms"])[:, None], c["prec"],
                                                   path="split")
                assert int(n[0]) == c["L"] and data[0].hex() == c["bytes"], (r.dtype, c)
                cd.close()


def test_kat1_identity_static_model():
    """KAT-1 on the GPU: uniform-256 static table (stride 0), prec 48, 1 MiB -> identity."""
    kat = load_golden("kat.json")["kat1"]
    data = np.random.default_rng(0).integers(0, 256, kat["n"], dtype=np.uint8)
    c = _coder(256, 1, 48, cap=kat["n"] * 8 + 4096)
    row = torch.ones(256, dtype=torch.int32, device=DEV)
    sym = torch.from_numpy(data.astype(np.int32)).to(DEV).view(-1, 1)
    c.encode(row, sym)
    c.finish()
    out, n = c.to_bytes()
    assert len(out[0]) == kat["out_len"] and hashlib.sha256(out[0]).hexdigest() == kat["out_sha256"]
    c.decode_open()
    dec = c.decode(row.view(1, 1, 256).expand(kat["n"], 1, 256)).cpu().numpy()[:, 0]
    assert bytes(dec.astype(np.uint8)) == data.tobytes()


# ---------------------------------------------------------------- batches vs oracle
BATCH_CASES = [
    # V, streams, steps, prec, kind
    (256, 64, 40, 24, "loguniform"),
    (1000, 96, 24, 48, "zeros"),
    (1000, 64, 16, 16, "loguniform"),      # fudged rows
    (300, 64, 32, 10, "flat"),             # mixed fudged / unfudged
    (1001, 33, 12, 48, "peaked"),          # odd V: scalar load path
    (3000, 40, 8, 61, "loguniform"),
    (1000, 32, 12, 48, "llama64"),         # u64 tables, every row fudged
    (32000, 16, 4, 48, "loguniform"),
    (32000, 8, 3, 24, "loguniform"),       # fudged at full vocab
]


@pytest.mark.parametrize("path,job", [("split", False), ("fused", False), ("fused", True), ("split", True)])
@pytest.mark.parametrize("V,B,steps,prec,kind", BATCH_CASES)
def test_batch_vs_oracle(V, B, steps, prec, kind, path, job):
    from oracle import oracle as coracle
    pmf, sym = synth.make_batch(1000 + V + prec, steps, B, V, kind)
    c, dpmf, data, n, tr = _gpu_encode(pmf, sym, prec, path=path, job=job)
    out, nb, status, rc = coracle.encode_batch(pmf, sym, prec, nthreads=16)
    assert rc == 0
    for b in range(B):
        assert int(n[b]) == int(nb[b]), b
        assert data[b] == out[b, :(int(nb[b]) + 7) // 8].tobytes(), b
    dec = _decode_both(c, dpmf)
    assert (dec == sym).all()
    c.raise_on_error()


def test_decode_external_bits_from_oracle():
    """Decode bitstreams produced by the oracle (user-provided device buffers)."""
    from oracle import oracle as coracle
    V, B, steps, prec = 512, 48, 20, 32
    pmf, sym = synth.make_batch(77, steps, B, V, "zeros")
    out, nb, status, rc = coracle.encode_batch(pmf, sym, prec, nthreads=8)
    stride = (out.shape[1] + 7) // 8 * 8
    buf = np.zeros((B, stride), dtype=np.uint8)
    buf[:, :out.shape[1]] = out
    c = _coder(V, B, prec)
    bits = torch.from_numpy(buf).to(DEV)
    nbits = torch.from_numpy(nb.astype(np.int64)).to(DEV)
    for path in DECODE_PATHS:
        c.set_decode_path(path)
        c.decode_open(bits, nbits)
        dec = c.decode(_dev_pmf(pmf)).cpu().numpy()
        assert (dec == sym).all()


def test_incremental_encode_matches_one_shot():
    """Several lac_encode calls (chunks not multiple of 64) == one call."""
    V, B, steps, prec = 700, 20, 150, 40
    pmf, sym = synth.make_batch(5, steps, B, V, "loguniform")
    _, _, one, n1, _ = _gpu_encode(pmf, sym, prec)
    c = _coder(V, B, prec, cap=steps * (prec + 2) + 256)
    dp, ds = _dev_pmf(pmf), torch.from_numpy(sym).to(DEV)
    for a, b in ((0, 1), (1, 70), (70, 71), (71, 150)):
        c.encode(dp[a:b], ds[a:b].contiguous())
    c.finish()
    two, n2 = c.to_bytes()
    assert (n1 == n2).all() and one == two


# ---------------------------------------------------------------- headline shape
def test_headline_shape_softmax_tables():
    """V=32000, 4096 streams, random-softmax u32 tables: sampled oracle parity,
    full round trip, and size-independent properties."""
    from oracle import oracle as coracle
    V, B, steps, prec = 32000, 4096, 3, 48
    pmf, sym = synth.softmax_tables(steps, B, V, seed=1234, device=DEV)
    c = _coder(V, B, prec, cap=steps * (prec + 2) + 256)
    c.encode_job(pmf, sym)                 # AUTO: fused kernel at 4096 streams
    data, n = c.to_bytes()
    c2 = _coder(V, B, prec, cap=steps * (prec + 2) + 256)
    c2.set_path("split")
    c2.encode(pmf, sym)
    c2.finish()
    assert c2.to_bytes()[0] == data
    c2.close()
    sample = list(range(0, B, 97)) + [B - 1]
    sub = pmf[:, sample, :].cpu().numpy().view(np.uint32)
    out, nb, status, rc = coracle.encode_batch(sub, sym[:, sample].cpu().numpy(), prec, nthreads=16)
    assert rc == 0
    for i, b in enumerate(sample):
        assert data[b] == out[i, :(int(nb[i]) + 7) // 8].tobytes()
    for path in DECODE_PATHS:
        c.set_decode_path(path)
        c.decode_open()
        assert torch.equal(c.decode(pmf), sym)
    # every stream ends in the group_bits format: padding bits are zero
    for b in range(0, B, 7):
        L = int(n[b])
        if L % 8:
            assert data[b][-1] & ((1 << (8 - L % 8)) - 1) == 0


def test_c2_shape_one_stream_4096_steps():
    """SURVEY c2 at its own shape: V=32000, ONE stream, 4096 steps of random-softmax
    u32 tables (seeded, 524 MB).  Bytes == the C oracle; the symbols come back
    through AUTO and every decode path; the decoder's determined count equals what
    the reference's bit-serial run(bits, stop=0) emits (the C oracle's literal
    restatement of it, pinned to the reference's golden counts)."""
    from oracle import oracle as coracle
    V, B, steps, prec = 32000, 1, 4096, 48
    pmf, sym = synth.softmax_tables(steps, B, V, seed=2024, device=DEV)
    c = _coder(V, B, prec, cap=steps * (prec + 2) + 256)
    c.encode_job(pmf, sym)
    data, n = c.to_bytes()
    host = pmf[:, 0, :].cpu().numpy().view(np.uint32)
    hsym = sym[:, 0].cpu().numpy()
    out, nb, status, rc = coracle.encode_batch(host[:, None, :], hsym[:, None], prec, nthreads=1)
    assert rc == 0 and int(nb[0]) == int(n[0]) and out[0, :(int(nb[0]) + 7) // 8].tobytes() == data[0]
    for path in ("auto",) + DECODE_PATHS:
        c.set_decode_path(path)
        c.decode_open()
        assert torch.equal(c.decode(pmf), sym), path
    dec = coracle.decode_bitserial(host, data[0], int(n[0]), prec, max_out=steps + 64)
    assert dec[:steps] == hsym.tolist()
    # the decoder's own determined count over the stream and the reference's
    c.set_decode_path("auto")
    c.decode_open()
    extra = len(dec) - steps
    tail = torch.cat([pmf, pmf[-1:].expand(extra + 1, B, V)]) if extra >= 0 else pmf
    got = c.decode(tail.contiguous())
    assert int(c.determined()[0]) == len(dec)
    assert got[:len(dec), 0].cpu().tolist() == dec
    c.close()


def test_c4_shape_softmax_tables():
    """SURVEY c4 at full size (V=128256 Llama-3 vocab, 4096 streams, u32 rows of
    513 KB): fused and split encoders byte-identical, sampled streams bit-exact
    against the C oracle, every stream round-trips through the AUTO decoder and the
    per-step decoder, and the bit counts sum to the same total both ways."""
    from oracle import oracle as coracle
    V, B, steps, prec = 128256, 4096, 2, 48
    pmf, sym = synth.softmax_tables(steps, B, V, seed=4242, device=DEV)
    c = _coder(V, B, prec, cap=steps * (prec + 2) + 256)
    c.encode_job(pmf, sym)
    data, n = c.to_bytes()
    c2 = _coder(V, B, prec, cap=steps * (prec + 2) + 256)
    c2.set_path("split")
    c2.encode(pmf, sym)
    c2.finish()
    d2, n2 = c2.to_bytes()
    assert d2 == data and (n2 == n).all()
    c2.close()
    sample = list(range(0, B, 331)) + [B - 1]
    sub = pmf[:, sample, :].cpu().numpy().view(np.uint32)
    out, nb, status, rc = coracle.encode_batch(sub, sym[:, sample].cpu().numpy(), prec, nthreads=16)
    assert rc == 0
    for i, b in enumerate(sample):
        assert int(n[b]) == int(nb[i]) and data[b] == out[i, :(int(nb[i]) + 7) // 8].tobytes(), b
    for path in ("auto", "split"):
        c.set_decode_path(path)
        c.decode_open()
        assert torch.equal(c.decode(pmf), sym), path
    c.close()


def test_c5_stream_count_on_one_gpu():
    """SURVEY c5's whole job -- V=128256, 32768 streams (8 x 4096) -- on one MI355X
    (2 steps: 33.6 GB of u32 rows, and the same shape as bf16 logits): sampled
    streams bit-exact against the C oracle, every stream round-trips, and the bits
    of stream b do not depend on the batch it is coded in (the first 4096 streams
    coded alone give the same bytes -- what lets c5 shard over 8 GPUs)."""
    from oracle import oracle as coracle
    V, B, steps, prec = 128256, 32768, 2, 48
    pmf, sym = synth.softmax_tables(steps, B, V, seed=55, device=DEV)
    c = _coder(V, B, prec, cap=steps * (prec + 2) + 256)
    c.encode_job(pmf, sym)
    data, n = c.to_bytes()
    sample = list(range(0, B, 2999)) + [B - 1]
    sub = pmf[:, sample, :].cpu().numpy().view(np.uint32)
    out, nb, status, rc = coracle.encode_batch(sub, sym[:, sample].cpu().numpy(), prec, nthreads=16)
    assert rc == 0
    for i, b in enumerate(sample):
        assert int(n[b]) == int(nb[i]) and data[b] == out[i, :(int(nb[i]) + 7) // 8].tobytes(), b
    c.decode_open()
    assert torch.equal(c.decode(pmf), sym)
    c.close()
    shard = _coder(V, 4096, prec, cap=steps * (prec + 2) + 256)
    shard.encode_job(pmf[:, 4096:8192], sym[:, 4096:8192].contiguous())
    assert shard.to_bytes()[0] == data[4096:8192]
    shard.close()
    del pmf
    c = _coder(V, B, prec, cap=steps * (prec + 2) + 256)
    lg, sym2 = synth.logits_batch(steps, B, V, seed=56, device=DEV, dtype=torch.bfloat16,
                                  quantise=c.quantize_logits)
    c.encode_logits_job(lg, sym2)
    data2, n2 = c.to_bytes()
    host = lg[:, sample, :].contiguous().view(torch.int16).cpu().numpy().view(np.uint16)
    out, nb, status, rc = coracle.encode_batch(coracle.q1_quantize(host, prec), sym2[:, sample].cpu().numpy(), prec,
                                               nthreads=16)
    assert rc == 0
    for i, b in enumerate(sample):
        assert int(n2[b]) == int(nb[i]) and data2[b] == out[i, :(int(nb[i]) + 7) // 8].tobytes(), b
    c.decode_open()
    assert torch.equal(c.decode_logits(lg), sym2)
    c.close()


# ---------------------------------------------------------------- errors
@pytest.mark.parametrize("path", ["split", "fused"])
def test_error_symbol_range(path):
    V, B = 16, 4
    pmf = torch.ones((2, B, V), dtype=torch.int32, device=DEV)
    sym = torch.zeros((2, B), dtype=torch.int32, device=DEV)
    sym[1, 2] = V          # AssertionError('unknown symbol', V) in the reference
    sym[0, 3] = -1
    c = _coder(V, B, 16)
    c.set_path(path)
    c.encode(pmf, sym)
    rc, err, step = c.status()
    assert rc != 0
    assert err.tolist() == [0, 0, -3, -3] and step[2] == 1 and step[3] == 0


@pytest.mark.parametrize("path", ["split", "fused"])
def test_error_zero_width_and_table(path):
    V, B = 8, 3
    pmf = torch.ones((1, B, V), dtype=torch.int32, device=DEV)
    pmf[0, 0, 5] = 0
    pmf[0, 1, :] = 0
    sym = torch.full((1, B), 5, dtype=torch.int32, device=DEV)
    c = _coder(V, B, 16)
    c.set_path(path)
    c.encode(pmf, sym)
    rc, err, step = c.status()
    assert err.tolist() == [-4, -5, 0]


@pytest.mark.parametrize("path", ["split", "fused"])
def test_error_capacity(path):
    V, B, steps = 1000, 2, 200
    pmf, sym = synth.make_batch(9, steps, B, V, "loguniform")
    c = _coder(V, B, 48, cap=128)
    c.set_path(path)
    c.encode(_dev_pmf(pmf), torch.from_numpy(sym).to(DEV))
    rc, err, step = c.status()
    assert (err == -7).all()


def test_open_rejects_bad_prec():
    from lac_amd._lib import LacError
    with pytest.raises(LacError):
        _coder(300, 1, 8)          # 2^(8-1) < 300: the reference coder hangs
    with pytest.raises(LacError):
        _coder(10, 1, 62)


# ---------------------------------------------------------------- run(bits, stop=0) counts
def _determined_case(rows, syms, extra, count, prec, data, L):
    """Decode len(syms)+len(extra)+2 steps (rows past the end repeat the last row,
    as the reference's Replay predictor does) and compare the determined count."""
    V = len(rows[0])
    n = len(syms) + len(extra) + 2
    tab = np.stack([np.asarray(rows[min(i, len(rows) - 1)], dtype=np.uint64) for i in range(n)])
    stride = ((len(data) + 7) // 8 + 1) * 8
    buf = np.zeros((1, stride), dtype=np.uint8)
    buf[0, :len(data)] = np.frombuffer(data, dtype=np.uint8)
    c = _coder(V, 1, prec, bits=64)
    out = {}
    for path in DECODE_PATHS:
        c.set_decode_path(path)
        c.decode_open(torch.from_numpy(buf).to(DEV), torch.tensor([L], dtype=torch.int64, device=DEV))
        dec = c.decode(torch.from_numpy(tab.view(np.int64).reshape(n, 1, V)).to(DEV)).cpu().numpy()[:, 0]
        nd = int(c.determined()[0])
        assert nd == count, (path, nd, count)
        assert dec[:count].tolist() == (list(syms) + list(extra))[:count]
        out[path] = nd
    c.close()
    return out


def test_determined_count_matches_reference_small():
    for kind in ("static", "perstep"):
        for c in load_golden("small_cases.json")[kind]:
            if not c["syms"] or "decoded_count" not in c:
                continue
            _determined_case(c["rows"], c["syms"], c["decoded_extra"], c["decoded_count"], c["prec"],
                             bytes.fromhex(c["bytes"]), c["L"])


@pytest.mark.parametrize("case", [c for c in load_golden("gen_cases.json") if "decoded_count" in c],
                         ids=lambda c: c["name"])
def test_determined_count_matches_reference_gen(case):
    rows = [synth.pmf_row(case["seed"], t, 0, case["V"], case["kind"], case["exp_range"]) for t in range(case["steps"])]
    _determined_case(rows, case["syms"], case["decoded_extra"], case["decoded_count"], case["prec"],
                     bytes.fromhex(case["bytes"]), case["L"])


# ---------------------------------------------------------------- edge cases
@pytest.mark.parametrize("path", ["split", "fused"])
def test_edge_single_symbol_alphabet(path):
    """V=1: every symbol is certain, no bits are emitted (as the reference)."""
    from oracle import restate
    c = _coder(1, 3, 16)
    c.set_path(path)
    pmf = torch.full((5, 3, 1), 7, dtype=torch.int32, device=DEV)
    sym = torch.zeros((5, 3), dtype=torch.int32, device=DEV)
    c.encode_job(pmf, sym)
    data, n = c.to_bytes()
    want, L = restate.encode_bytes([[7]], [0] * 5, 16)
    assert all(d == want for d in data) and (n == L).all()
    c.decode_open()
    assert torch.equal(c.decode(pmf), sym)


@pytest.mark.parametrize("prec,V", [(2, 2), (3, 4), (10, 512), (11, 1024), (17, 65536)])
def test_edge_vocab_at_precision_boundary(prec, V):
    """2^(prec-1) == V (the largest vocabulary a precision admits) and tiny precisions."""
    from oracle import oracle as coracle
    pmf, sym = synth.make_batch(prec * 7 + V, 12, 5, V, "flat")
    c, dpmf, data, n, tr = _gpu_encode(pmf, sym, prec)
    out, nb, status, rc = coracle.encode_batch(pmf, sym, prec, nthreads=4)
    assert rc == 0
    for b in range(5):
        assert data[b] == out[b, :(int(nb[b]) + 7) // 8].tobytes()
    assert (_decode_both(c, dpmf) == sym).all()


@pytest.mark.parametrize("path", ["split", "fused"])
def test_edge_zero_steps_job(path):
    """A job with no symbols flushes the initial interval only (A_to_bin().run([]))."""
    from oracle import restate
    c = _coder(10, 4, 20)
    c.set_path(path)
    pmf = torch.ones((0, 4, 10), dtype=torch.int32, device=DEV)
    sym = torch.zeros((0, 4), dtype=torch.int32, device=DEV)
    c.encode_job(pmf, sym)
    data, n = c.to_bytes()
    want, L = restate.encode_bytes([[1] * 10], [], 20)
    assert all(d == want for d in data) and (n == L).all()


def test_edge_ragged_streams_and_extreme_tables():
    """Streams of very different entropy in one batch (one near-deterministic, one
    uniform, one with a 2^31 spike) end at different lengths; all bit-exact."""
    from oracle import oracle as coracle
    V, B, T, prec = 4096, 6, 40, 48
    rng = np.random.default_rng(5)
    pmf = np.ones((T, B, V), dtype=np.uint32)
    pmf[:, 0, 17] = 2 ** 31                      # near-certain symbol 17
    pmf[:, 2, :] = rng.integers(1, 2 ** 31, (T, V), dtype=np.uint32)
    pmf[:, 3, ::2] = 0                           # half the alphabet impossible
    pmf[:, 4, :] = 0
    pmf[:, 4, 100:102] = 2 ** 31 - 1             # two-symbol row
    pmf[:, 5, :] = 2 ** 32 - 1                   # maximal entries everywhere
    sym = rng.integers(0, V, (T, B)).astype(np.int32)
    sym[:, 0] = 17
    sym[:, 3] = (sym[:, 3] // 2) * 2 + 1
    sym[:, 4] = 100 + (sym[:, 4] & 1)
    c, dpmf, data, n, tr = _gpu_encode(pmf, sym, prec)
    out, nb, status, rc = coracle.encode_batch(pmf, sym, prec, nthreads=6)
    assert rc == 0
    assert len(set(int(x) for x in n)) >= 4
    for b in range(B):
        assert data[b] == out[b, :(int(nb[b]) + 7) // 8].tobytes(), b
    assert (_decode_both(c, dpmf) == sym).all()


def test_edge_u64_total_overflow_is_an_error():
    V, B = 8, 2
    pmf = np.full((1, B, V), 2 ** 62, dtype=np.uint64)      # total 2^65
    pmf[0, 1, :] = 1
    sym = np.zeros((1, B), dtype=np.int32)
    c = _coder(V, B, 48, bits=64)
    c.encode(_dev_pmf(pmf), torch.from_numpy(sym).to(DEV))
    rc, err, step = c.status()
    assert err.tolist() == [-5, 0]


@pytest.mark.parametrize("path", ["split", "fused"])
def test_edge_u64_totals_near_2_63(path):
    """u64 rows whose totals straddle 2^63: below it the split path's coder step
    divides through row fractions, from it on (no fraction fits) it falls back to
    the quotient estimates -- both bit-exact vs the oracle, at prec 61 where w
    reaches 2^61, with zero entries and unfudged / fudged rows mixed."""
    from oracle import oracle as coracle
    rng = np.random.default_rng(63)
    V, B, steps, prec = 6, 12, 40, 61
    pmf = np.zeros((steps, B, V), dtype=np.uint64)
    for b in range(B):
        hi = (1 << 63) // V * (40 + b - 3) // 40                # totals just below / above 2^63
        pmf[:, b, :] = rng.integers(hi // 8 * 7, hi, size=(steps, V), dtype=np.uint64)
    pmf[::7, :, 2] = 0                                          # zero-probability entries
    pmf[::3, ::3, 5] = 1                                        # minp 1: those rows take fudged_dist
    sym = rng.integers(0, V, size=(steps, B)).astype(np.int32)
    sym[::7][sym[::7] == 2] = 3
    tot = pmf.astype(object).sum(axis=2)
    assert (tot < (1 << 64)).all() and (tot >= (1 << 63)).any() and (tot < (1 << 63)).any()
    c, dpmf, data, n, tr = _gpu_encode(pmf, sym, prec, path=path)
    out, nb, status, rc = coracle.encode_batch(pmf, sym, prec, nthreads=4)
    assert rc == 0
    for b in range(B):
        assert int(n[b]) == int(nb[b]) and data[b] == out[b, :(int(nb[b]) + 7) // 8].tobytes(), b
    assert (_decode_both(c, dpmf) == sym).all()


@pytest.mark.gpu
@pytest.mark.parametrize("prec", [48, 61])
def test_edge_u64_totals_near_2_62(prec):
    """The split path's compare-free row-fraction quotients (frac_mul_div<true>: sign
    masks of r - T and r - 2T, valid for totals below 2^62) and, from 2^62 on, the
    divisions k_encode falls back to: u64 rows whose totals straddle 2^62, few streams
    (k_encode's uniform chain), fudged rows mixed in; bit-exact vs the oracle."""
    from oracle import oracle as coracle
    rng = np.random.default_rng(62)
    V, B, steps = 6, 12, 40
    pmf = np.zeros((steps, B, V), dtype=np.uint64)
    for b in range(B):
        hi = (1 << 62) // V * (36 + b) // 40                    # totals from ~0.8 to ~1.2 x 2^62
        pmf[:, b, :] = rng.integers(hi // 8 * 7, hi, size=(steps, V), dtype=np.uint64)
    pmf[::3, ::3, 5] = 1                                        # minp 1: fudged_dist at these totals
    sym = rng.integers(0, V, size=(steps, B)).astype(np.int32)
    tot = pmf.astype(object).sum(axis=2)
    assert (tot >= (1 << 62)).any() and (tot < (1 << 62)).any()
    c, dpmf, data, n, tr = _gpu_encode(pmf, sym, prec, path="split")
    out, nb, status, rc = coracle.encode_batch(pmf, sym, prec, nthreads=4)
    assert rc == 0
    for b in range(B):
        assert int(n[b]) == int(nb[b]) and data[b] == out[b, :(int(nb[b]) + 7) // 8].tobytes(), b
    assert (_decode_both(c, dpmf) == sym).all()


def test_stats_decode_spans_step_chunks():
    """600 streams x 150 steps: the stats-path decode (AUTO below 2048 streams)
    runs in 64-step chunks; symbols and determined counts match the other paths."""
    V, B, steps, prec = 512, 600, 150, 40
    pmf, sym = synth.make_batch(21, steps, B, V, "loguniform")
    c, dpmf, data, n, tr = _gpu_encode(pmf, sym, prec)
    dets = []
    for path in DECODE_PATHS:
        c.set_decode_path(path)
        c.decode_open()
        assert (c.decode(dpmf).cpu().numpy() == sym).all(), path
        dets.append(c.determined())
    assert all((d == dets[0]).all() for d in dets[1:])
    c.raise_on_error()


# ------------------------------------------------- one-wave decode granularity
@pytest.mark.gpu
@pytest.mark.parametrize("V,bits", [(32000, 32), (32004, 32), (32768, 32), (33024, 32), (65540, 32),
                                    (128256, 32), (131076, 32), (16000, 64), (32000, 64), (65538, 64)])
def test_decode_wave_granularity(V, bits):
    """k_decode_wave_fine (per-iteration totals; register counts 2/4/8 and the
    fallback beyond 512 iterations) against the chunk-total kernel, the per-step
    kernel and the symbols, on ragged and exact row lengths, u32 and unfudged u64."""
    from oracle import oracle as coracle
    B, steps, prec = 16, 3, 48
    pmf, sym = synth.softmax_tables(steps, B, V, seed=77 + V, device=DEV)
    if bits == 64:
        pmf = pmf.to(torch.int64)
    c = _coder(V, B, prec, bits=bits, cap=steps * (prec + 2) + 256)
    c.encode_job(pmf, sym)
    data, n = c.to_bytes()
    host = pmf[:, :4, :].cpu().numpy()
    host = host.view(np.uint32) if bits == 32 else host.view(np.uint64)
    out, nb, _, rc = coracle.encode_batch(host, sym[:, :4].cpu().numpy(), prec, nthreads=4)
    assert rc == 0
    for b in range(4):
        assert data[b] == out[b, :(int(nb[b]) + 7) // 8].tobytes()
    for path in ("fused", "fused_chunk", "split", "block", "stats"):
        c.set_decode_path(path)
        c.decode_open()
        assert torch.equal(c.decode(pmf), sym), path
    for nw in (4, 8, 16):
        c.set_decode_path("block")
        c.set_block_waves(nw)
        c.decode_open()
        assert torch.equal(c.decode(pmf), sym), nw
    c.close()


@pytest.mark.parametrize("prec", [20, 33, 34, 48])
def test_edge_u64_large_entries_minp_beyond_32_bits(prec):
    """u64 rows whose smallest positive entry is >= 2^32: the decoders find minp
    with 32-bit keys, so such rows take the exact 64-bit re-scan exactly when the
    fudge test could flip (T > w * 2^32, below prec 34).  Fudged and unfudged
    rows, every decode path, against the C oracle."""
    from oracle import oracle as coracle
    rng = np.random.default_rng(prec)
    V, B, steps = 16, 8, 12
    pmf = rng.integers(1 << 32, 1 << 40, size=(steps, B, V), dtype=np.uint64)
    pmf[:, ::2, 3] = rng.integers(1 << 58, 1 << 59, size=(steps, B // 2), dtype=np.uint64)
    pmf[::4, :, 5] = 0
    pmf[:, 1, 7] = (1 << 32) - 1                                 # minp just below 2^32
    sym = rng.integers(0, V, size=(steps, B)).astype(np.int32)
    sym[::4][sym[::4] == 5] = 6
    c, dpmf, data, n, tr = _gpu_encode(pmf, sym, prec)
    out, nb, status, rc = coracle.encode_batch(pmf, sym, prec, nthreads=4)
    assert rc == 0
    for b in range(B):
        assert int(n[b]) == int(nb[b]) and data[b] == out[b, :(int(nb[b]) + 7) // 8].tobytes(), b
    assert (_decode_both(c, dpmf) == sym).all()


def test_edge_u64_decode_total_at_2_64():
    """Decoding against u64 rows whose totals are 2^64 - 1 (valid), exactly 2^64
    with every high word summing below 2^32, and 2^64 + 5: the two overflowing
    streams fail with LAC_E_TABLE on every decode path (the wrapped-total test)."""
    V, B = 2, 3
    rows = [[0x7FFFFFFFFFFFFFFF, 0x8000000000000001],           # T = 2^64, high words 2^32 - 1
            [1 << 63, (1 << 63) - 1],                            # T = 2^64 - 1
            [(1 << 63) + 3, (1 << 63) + 2]]                      # T = 2^64 + 5
    pmf = np.array([rows], dtype=np.uint64)
    bits = torch.zeros((B, 16), dtype=torch.uint8, device=DEV)
    nbits = torch.full((B,), 64, dtype=torch.int64, device=DEV)
    for path in DECODE_PATHS:
        c = _coder(V, B, 48, bits=64)
        c.set_decode_path(path)
        c.decode_open(bits, nbits)
        out = c.decode(_dev_pmf(pmf)).cpu().numpy()
        rc, err, step = c.status()
        assert err.tolist() == [-5, 0, -5], path
        assert out[0].tolist()[0] == -1 and out[0].tolist()[2] == -1 and out[0].tolist()[1] >= 0, path
        c.close()
