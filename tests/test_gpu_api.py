"""The reference-shaped API (lac_amd.coder / lac_amd.sampler) on the GPU, against
vectors the reference produced (tests/golden)."""
import hashlib

import numpy as np
import pytest

from conftest import load_golden

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

MISC = load_golden("misc.json")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def test_ternary_docstring_example():
    """AC() = uniform ternary Predictor at prec 16 (arith_code.py:15-52, :143-145)."""
    from lac_amd.coder import AC
    t = MISC["ternary"]
    ac = AC()
    assert list(ac.to_bin.run([1, 1, 2])) == t["digits"]
    assert list(ac.to_bin.encode([1, 1, 2])) == t["encode"]
    assert list(ac.to_bin.bits([1, 1, 2])) == t["bits"]
    assert list(ac.from_bin.run(t["bits"], stop=0, n=3)) == t["decoded"]


def test_step_and_call_match_run():
    from lac_amd.coder import AC, CDFPredictor
    c = [c for c in load_golden("small_cases.json")["static"] if len(c["syms"]) >= 4][0]
    ac = AC(CDFPredictor(list(np.cumsum(c["rows"][0]).tolist())), c["prec"])
    enc = ac.to_bin
    steps = [enc(s) for s in c["syms"]]
    assert [list(x) for x in steps] == c["trace"]
    assert list(enc(None)) == c["flush"]


@pytest.mark.parametrize("kind", ["static", "perstep"])
def test_cdfpredictor_against_golden(kind):
    """CDFPredictor / Replay-style predictors through AC, for 40 reference cases."""
    from lac_amd.coder import AC, CDFPredictor, group_bits, measure_compress

    class Replay(CDFPredictor):
        def __init__(self, rows):
            self.rows, self.i = rows, 0
            self._load()

        def _load(self):
            self.dist = np.cumsum(self.rows[min(self.i, len(self.rows) - 1)]).tolist()
            self.minp = min(x for x in self.rows[min(self.i, len(self.rows) - 1)] if x > 0)

        def accept(self, s):
            self.i += 1
            self._load()

        def copy(self):
            return Replay(self.rows)

    cases = [c for c in load_golden("small_cases.json")[kind] if c["syms"]][:40]
    makers = [lambda c: Replay(c["rows"])]
    if kind == "static":            # a plain CDFPredictor: the static-model (stride-0) paths
        makers.append(lambda c: CDFPredictor(np.cumsum(np.asarray(c["rows"][0], dtype=object)).tolist()))
    for mk in makers:
        for c in cases:
            ac = AC(mk(c), c["prec"])
            R, L = ac.to_bin.encode(c["syms"])
            assert L == c["L"] and R == int(c["bytes"] or "0", 16) >> ((-L) % 8)
            data = measure_compress(ac.to_bin, iter(c["syms"]), print_every_inp=1 << 30, print_every_out=1 << 30)
            assert data.hex() == c["bytes"]
            bits = list(ac.to_bin.bits(c["syms"]))
            assert bytes(group_bits(iter(bits))).hex() == c["bytes"]
            digits = list(ac.to_bin.run(c["syms"]))
            assert digits == [d for st in c["trace"] for d in st] + c["flush"]
            assert list(ac.from_bin.run(bits, stop=0, n=len(c["syms"]))) == c["syms"]
            # without n: exactly what the reference's bit-serial run(bits, stop=0) emits
            assert list(ac.from_bin.run(bits, stop=0)) == c["syms"] + c["decoded_extra"]


def test_bit_serial_step_matches_reference():
    """A_from_bin.step(bit) / __call__(bit) (arith_code.py:291-298, 318-321): after
    every bit, exactly the symbols the reference's step(bit) yields -- per-bit counts
    recorded by running the reference over 77 golden streams (tests/golden/
    step_cases.json, tools/gen_golden_step.py): static and per-step tables, V up to
    1000, prec 10..61, fudged rows included."""
    from lac_amd import synth
    from lac_amd.coder import AC, CDFPredictor

    class Replay(CDFPredictor):
        def __init__(self, rows):
            self.rows, self.i = rows, 0
            self._load()

        def _load(self):
            r = self.rows[min(self.i, len(self.rows) - 1)]
            self.dist = np.cumsum(np.asarray(r, dtype=object)).tolist()
            self.minp = min(int(x) for x in r if x > 0)

        def accept(self, s):
            self.i += 1
            self._load()

    gen = {c["name"]: c for c in load_golden("gen_cases.json")}
    for case in load_golden("step_cases.json")["cases"]:
        if "rows" in case:
            rows = case["rows"]
        else:
            g = gen[case["gen"]]
            rows = [synth.pmf_row(g["seed"], t, 0, g["V"], g["kind"], g["exp_range"]).tolist()
                    for t in range(g["steps"])]
        data = bytes.fromhex(case["bytes"])
        bits = [(data[i >> 3] >> (7 - (i & 7))) & 1 for i in range(case["L"])]
        dec = AC(Replay(rows), case["prec"]).from_bin
        counts, syms = [], []
        for i, b in enumerate(bits):
            out = dec(b) if i % 2 else tuple(dec.step(b))
            counts.append(len(out))
            syms.extend(out)
        assert counts == case["counts"], case["src"]
        assert syms == case["syms"], case["src"]
    # a longer stream (the bit buffer grows several times): step() == run(bits, stop=0)
    data = bytes(np.random.default_rng(9).integers(0, 256, 400, dtype=np.uint8))
    ac = AC(CDFPredictor(list(range(1, 257))), 48)
    bits = list(ac.to_bin.bits(iter(data)))
    dec = AC(CDFPredictor(list(range(1, 257))), 48).from_bin
    stepped = [s for b in bits for s in dec.step(b)]
    assert stepped == list(ac.from_bin.run(bits, stop=0)) and bytes(stepped[:len(data)]) == data
    # the registers after each bit: l <= lb <= hb <= h once a symbol is out, and the
    # [lb, hb] interval halves per received bit as receive_bit does (:264-267)
    dec = AC(CDFPredictor(list(range(1, 257))), 48).from_bin
    assert (dec.l, dec.h, dec.lb, dec.hb) == (0, (1 << 48) - 1, 0, (1 << 48) - 1)
    for i, b in enumerate(bits[:300]):
        w = dec.hb - dec.lb + 1
        before = (dec.lb, dec.h - dec.l)
        out = list(dec.step(b))
        if not out:
            assert dec.hb - dec.lb + 1 == w // 2 and dec.lb == before[0] + b * (w // 2)
        assert dec.l <= dec.lb <= dec.hb <= dec.h or not out
    assert repr(dec).startswith("A_from_bin([")
    # lac_decode_set_state refuses registers no decoder reaches (nothing is copied)
    import ctypes as C
    from lac_amd._lib import LacError, check
    c = dec._sess.coder
    st = dec._sess.st.copy()
    for field, bad in (("l", -1), ("h", -5), ("pos", 3)):
        b = st.copy()
        b[field] = bad
        with pytest.raises(LacError):
            check(c.lib.lac_decode_set_state(c.ctx, b.ctypes.data_as(C.c_void_p), c._stream))
    b = st.copy()
    b["h"] = int(b["l"][0]) + (1 << 48)
    with pytest.raises(LacError):
        check(c.lib.lac_decode_set_state(c.ctx, b.ctypes.data_as(C.c_void_p), c._stream))
    # run() on a decoder that step() has fed continues it, as the reference's run does
    dec = AC(CDFPredictor(list(range(1, 257))), 48).from_bin
    head = [s for b in bits[:1000] for s in dec.step(b)]
    assert head + list(dec.run(bits[1000:], stop=0)) == stepped


def test_probpredictor_subclass_adaptive():
    """An adaptive ProbPredictor (counts of past symbols) round-trips and matches the oracle."""
    from lac_amd.coder import AC, ProbPredictor
    from oracle import restate

    class Counts(ProbPredictor):
        def __init__(self, n, counts=None):
            super().__init__(n)
            self.counts = list(counts) if counts else [1] * n

        def prob(self, s):
            return self.counts[s] * 1000 + 1

        def accept(self, s):
            self.counts[s] += 1
            super().accept(s)

        def copy(self):
            return Counts(self.n, self.counts)

    rng = np.random.default_rng(4)
    syms = rng.integers(0, 7, 300).tolist()
    ac = AC(Counts(7), 24)
    bits = list(ac.to_bin.bits(syms))
    p = Counts(7)
    rows = []
    for s in syms:
        rows.append([p.prob(i) for i in range(7)])
        p.accept(s)
    want, L = restate.encode_bytes(rows, syms, 24)
    assert len(bits) == L and bytes(restate.group_bits(bits)) == want
    assert list(ac.from_bin.run(bits, stop=0, n=len(syms))) == syms


def test_symbol_range_raises_like_reference():
    from lac_amd.coder import AC, CDFPredictor
    ac = AC(CDFPredictor([1, 3, 6, 10]), 16)
    with pytest.raises(AssertionError) as e:
        list(ac.to_bin.run([0, 4]))
    assert e.value.args[0] == "unknown symbol" and e.value.args[1] == 4


def test_acsampler_small_sampler_api():
    """ACSampler(48) loop over np.ones(256), 1000 bytes."""
    from lac_amd.sampler import ACSampler, packbits
    k = MISC["acsampler_small"]
    data = np.random.default_rng(0).integers(0, 256, k["n"], dtype=np.uint8)
    out = bytearray()
    s = ACSampler(48)
    s.compress_tokens = iter(data.tolist())
    s.compress_output = packbits(out.append)

    def done():
        s.on_compress_done = None
        s.flush_compress()
        s.compress_output.flush()
        s.compress_output = None
    s.on_compress_done = done
    while not s.compress_done:
        s.sample(np.ones(256))
    assert bytes(out).hex() == k["out_hex"]


def test_acsampler_nonuniform_golden():
    from lac_amd.sampler import encode_acsampler
    for c in MISC["acsampler_nonuniform"]:
        cdf = np.array(c["cdf"], dtype=np.uint64)
        pmf = np.concatenate([cdf[:1], np.diff(cdf)])
        bits = encode_acsampler([pmf] * len(c["tokens"]), c["tokens"], 48)
        assert "".join(map(str, bits)) == c["bits"]


def test_kat2_acsampler_gpu():
    """KAT-2: ACSampler uniform-256 encode of 1 MiB = input || 0x00 (reference-verified hash)."""
    from lac_amd.sampler import encode_acsampler
    from oracle import restate
    kat = load_golden("kat.json")["kat2"]
    data = np.random.default_rng(0).integers(0, 256, kat["n"], dtype=np.uint8)
    cdf = restate.acsampler_cdf(np.ones(256))
    pmf = np.concatenate([cdf[:1], np.diff(cdf)]).astype(np.uint64)
    bits = encode_acsampler([pmf] * kat["n"], data.tolist(), 48)
    out = bytes(restate.group_bits(bits))
    assert len(out) == kat["out_len"] and hashlib.sha256(out).hexdigest() == kat["out_sha256"]


def test_container_compress_decompress_batch():
    from lac_amd import container, synth
    from lac_amd.batch import BatchCoder
    pmf, sym = synth.softmax_tables(6, 300, 2000, seed=7, device="cuda:0")
    coder = BatchCoder(2000, 300, prec=48, capacity_bits=6 * 50 + 256, device="cuda:0")
    blob = container.compress_batch(coder, pmf, sym)
    out, n = container.decompress_batch(blob, pmf)
    assert n == [6] * 300 and torch.equal(out, sym)


def test_container_logits_roundtrip():
    """A q1 container: bf16 logits in, flag set, decode with the same logits."""
    from lac_amd import container, synth
    from lac_amd.batch import BatchCoder
    coder = BatchCoder(2048, 300, prec=48, capacity_bits=6 * 50 + 256, device="cuda:0")
    logits, sym = synth.logits_batch(6, 300, 2048, seed=8, device="cuda:0", quantise=coder.quantize_logits)
    blob = container.compress_batch(coder, logits, sym)
    assert container.unpack(blob)["q1_logits"]
    out, n = container.decompress_batch(blob, logits)
    assert n == [6] * 300 and torch.equal(out, sym)
    with pytest.raises(ValueError):
        container.decompress_batch(blob, coder.quantize_logits(logits))


def test_llama_ac_adapter_with_torch_model_roundtrip():
    """Llama_AC (llama_compress.py:14-61) driven by a ROCm torch model: encode, decode,
    and bit-exact against the oracle on the tables the model produced."""
    from lac_amd.coder import AC, group_bits
    from lac_amd.llm import Llama_AC, TinyCausalLM, TorchLLM
    from oracle import restate
    V = 2000
    llm = TorchLLM(TinyCausalLM(vocab=V, d=32, layers=1, heads=2, max_len=64), n_ctx=24, device="cuda:0")
    rng = np.random.default_rng(11)
    toks = rng.integers(0, V, 40).tolist()           # crosses the n_ctx sliding window
    ac = AC(Llama_AC(llm), 48)
    bits = list(ac.to_bin.bits(toks))
    # replay the same model to get the integer rows, encode them with the oracle
    p = Llama_AC(llm)
    rows = []
    for t in toks:
        rows.append([int(x) for x in p.pmf_row()])
        p.accept(t)
    want, L = restate.encode_bytes(rows, toks, 48)
    assert len(bits) == L and bytes(group_bits(iter(bits))) == want
    assert list(ac.from_bin.run(bits, stop=0, n=len(toks))) == toks


@pytest.mark.parametrize("incremental", [True, False])
def test_logits_compressor_roundtrip_and_oracle(incremental):
    """LLM compression through the logits path, bf16 logits straight into the coder:
    incremental (TinyCausalLM's key/value-cache steps on both sides, O(T)) and, for a
    module with only forward(), one teacher-forced forward + fixed-shape decode
    forwards.  Bytes == q1 oracle + encode oracle on the logits compress coded with;
    decompress reproduces the tokens."""
    from lac_amd.llm import LogitsCompressor, TinyCausalLM
    from oracle import oracle as coracle
    V, B, T, prec = 1024, 4, 24, 48
    model = TinyCausalLM(vocab=V, d=32, layers=1, heads=2, max_len=64)
    if not incremental:
        class Plain(torch.nn.Module):                          # forward() only: no cache
            def __init__(self):
                super().__init__()
                self.m = model

            def forward(self, x):
                return self.m(x)
        model = Plain()
    lc = LogitsCompressor(model, V, prec=prec, device="cuda:0")
    assert lc.incremental == incremental
    toks = torch.from_numpy(np.random.default_rng(5).integers(0, V, (B, T))).to("cuda:0")
    data, nbits = lc.compress(toks)
    lg = lc.logits(toks)                                        # [B, T, V] bf16, as compress saw it
    host = lg.transpose(0, 1).contiguous().view(torch.int16).cpu().numpy().view(np.uint16)
    pmf = coracle.q1_quantize(host, prec)
    out, nb, status, rc = coracle.encode_batch(pmf, toks.t().contiguous().cpu().numpy().astype(np.int32), prec)
    assert rc == 0
    for b in range(B):
        assert int(nbits[b]) == int(nb[b]) and data[b] == out[b, :(int(nb[b]) + 7) // 8].tobytes()
    back = lc.decompress(data, nbits, T)
    assert torch.equal(back, toks)


def test_logits_compressor_vocab_not_a_multiple_of_8():
    """A vocab the 16-B row vectors do not divide (1001, bf16 and f32): rows padded
    with -inf, bytes == oracle on the padded logits, tokens round trip, and the
    library itself refuses the unpadded rows (LAC_E_ARG)."""
    from lac_amd._lib import LacError
    from lac_amd.batch import BatchCoder, pad_logits
    from lac_amd.llm import LogitsCompressor, TinyCausalLM
    from oracle import oracle as coracle
    V, B, T, prec = 1001, 3, 12, 48
    model = TinyCausalLM(vocab=V, d=32, layers=1, heads=2, max_len=64, seed=4)
    toks = torch.from_numpy(np.random.default_rng(6).integers(0, V, (B, T))).to("cuda:0")
    for dt in (torch.bfloat16, torch.float32):
        lc = LogitsCompressor(model, V, prec=prec, logits_dtype=dt, device="cuda:0")
        assert lc.vcode == (1008 if dt == torch.bfloat16 else 1004)
        data, nbits = lc.compress(toks)
        lg = lc.logits(toks)
        assert lg.shape[-1] == lc.vcode and torch.isinf(lg[..., V:]).all()
        h = lg.transpose(0, 1).contiguous()
        host = h.view(torch.int16).cpu().numpy().view(np.uint16) if dt == torch.bfloat16 else h.cpu().numpy()
        pmf = coracle.q1_quantize(host, prec)
        assert (pmf[..., V:] == 1).all()
        out, nb, status, rc = coracle.encode_batch(pmf, toks.t().contiguous().cpu().numpy().astype(np.int32), prec)
        assert rc == 0
        for b in range(B):
            assert int(nbits[b]) == int(nb[b]) and data[b] == out[b, :(int(nb[b]) + 7) // 8].tobytes()
        assert torch.equal(lc.decompress(data, nbits, T), toks)
        raw = torch.randn((T, B, V), device="cuda:0").to(dt)
        c = BatchCoder(V, B, prec=prec, device="cuda:0")
        with pytest.raises(LacError):
            c.encode_logits_job(raw, toks.t().contiguous().to(torch.int32))
        c.close()
        assert pad_logits(raw).shape[-1] == lc.vcode


@pytest.mark.parametrize("case", load_golden("llama_cases.json")["cases"], ids=lambda c: c["name"])
def test_llama_ac_bits_match_reference_fixture(case):
    """AC(lac_amd Llama_AC(llm), 48) on the GPU == the reference's A_to_bin on the
    CDFs the reference's own Llama_AC computed (exact ints), for a fake llm whose
    sliding window wraps (tests/golden/llama_cases.json, tools/gen_golden_llama.py);
    the decoder returns the tokens."""
    from fake_llm import FakeLlama
    from lac_amd.coder import AC, group_bits
    from lac_amd.llm import Llama_AC
    llm = FakeLlama(case["vocab"], case["n_ctx"], case["seed"], scale=case.get("scale", 3.0))
    ac = AC(Llama_AC(llm), case["prec"])
    bits = list(ac.to_bin.bits(case["tokens"]))
    assert len(bits) == case["exact_L"] and bytes(group_bits(iter(bits))).hex() == case["exact_bytes"]
    assert list(ac.from_bin.run(bits, stop=0, n=len(case["tokens"]))) == case["tokens"]


@pytest.mark.parametrize("case", load_golden("llama_cases.json")["refuse"], ids=lambda c: c["name"])
def test_llama_ac_refuses_rows_whose_fudge_decision_differs(case):
    """Rows where the reference's minp (0: zero CDF steps) and the table's smallest
    positive entry (>= 2^12) give different fudged_dist decisions at some width
    (tests/golden/llama_cases.json "refuse"): the GPU coder raises ValueError instead
    of coding bits that differ from the reference's."""
    from fake_llm import HeadLlama
    from lac_amd.coder import AC
    from lac_amd.llm import Llama_AC
    ac = AC(Llama_AC(HeadLlama(case["vocab"], case["n_ctx"], case["heads"], case["floor"])), case["prec"])
    with pytest.raises(ValueError, match="minp"):
        list(ac.to_bin.bits(case["tokens"]))


def _static_case(V=300, n=10000, seed=7):
    rng = np.random.default_rng(seed)
    pmf = rng.integers(1, 1000, V).astype(np.uint64)
    syms = rng.choice(V, size=n, p=pmf / pmf.sum()).tolist()
    return pmf, syms


def test_step_loop_10k_symbols_matches_oracle():
    """A_to_bin.step/__call__ one symbol at a time for 10k symbols (far beyond the
    first coder's capacity): digits == the C oracle's (capacity was
    sized by the cumulative emitted bits)."""
    from lac_amd.coder import AC, CDFPredictor
    from oracle import oracle as coracle
    pmf, syms = _static_case()
    prec = 48
    _, _, want = coracle.encode(pmf, syms, prec, static=True)
    enc = AC(CDFPredictor(np.cumsum(pmf).tolist()), prec).to_bin
    got = []
    for s in syms:
        got.extend(enc(s))
    got.extend(enc(None))
    assert got == want
    assert enc.emitted_bits == len(want)


def test_encoder_reuse_after_flush_longer_input():
    """run() again on a flushed encoder with a longer input (reference: the coder
    restarts from l=0, h=2^prec-1 after flush, arith_code.py:193-202)."""
    from lac_amd.coder import AC, CDFPredictor
    from oracle import oracle as coracle
    pmf, syms = _static_case(n=20000, seed=8)
    prec = 40
    enc = AC(CDFPredictor(np.cumsum(pmf).tolist()), prec).to_bin
    for n in (10, 3000, 20000, 5):
        _, _, want = coracle.encode(pmf, syms[:n], prec, static=True)
        assert list(enc.run(syms[:n])) == want, n


def test_run_then_steps_then_long_run_without_flush():
    """Mixing run(stop=0), step() and a long run() on one stream: the capacity is
    recovered by rebasing the device planes, the digits stay exact."""
    from lac_amd.coder import AC, CDFPredictor
    from oracle import restate
    pmf, syms = _static_case(V=50, n=12000, seed=9)
    prec = 32
    enc = AC(CDFPredictor(np.cumsum(pmf).tolist()), prec).to_bin
    got = list(enc.run(syms[:100], stop=0))
    for s in syms[100:200]:
        got.extend(enc.step(s))
    got.extend(enc.run(syms[200:], stop=1))
    assert got == restate.encode_digits([pmf.tolist()], syms, prec)


def test_silent_step_then_long_run_keeps_registers():
    """step() on a symbol of p > 1/2 narrows l, h without emitting a digit; a
    following run() longer than the first coder's capacity must continue those
    registers, not reallocate from l = 0."""
    from lac_amd.coder import AC, CDFPredictor
    from oracle import restate
    rng = np.random.default_rng(12)
    pmf = np.array([900] + rng.integers(1, 20, 15).tolist(), dtype=np.uint64)
    syms = [0] + rng.choice(16, size=3000, p=pmf / pmf.sum()).tolist()
    prec = 16
    enc = AC(CDFPredictor(np.cumsum(pmf).tolist()), prec).to_bin
    first = list(enc.step(0))
    assert first == [] and (enc.l, enc.h) != (0, (1 << prec) - 1)
    got = first + list(enc.run(syms[1:], stop=1))
    assert got == restate.encode_digits([pmf.tolist()], syms, prec)
    # a table-size change after a silent step is refused (the registers are live)
    enc = AC(CDFPredictor(np.cumsum(pmf).tolist()), prec).to_bin
    list(enc.step(0))
    enc.predictor = CDFPredictor(list(range(1, 9)))
    with pytest.raises(RuntimeError):
        list(enc.step(1))


def test_debug_log_matches_reference():
    """A_to_bin.debug_log (arith_code.py:164, 170, 182) of the GPU coder: the
    reference's (l, h, 'recv' | 'emit', x) entries for CDFPredictor encodes
    (tests/golden/custom_cases.json table_logs, tools/gen_golden_custom.py)."""
    from lac_amd.coder import AC, CDFPredictor
    for c in load_golden("custom_cases.json")["table_logs"]:
        enc = AC(CDFPredictor(c["cdf"]), c["prec"]).to_bin
        enc.debug_log = ["start"]                    # logged only into a truthy list, as there
        bits = list(enc.bits(c["syms"]))
        assert "".join(map(str, bits)) == c["bits"]
        assert [list(x) if isinstance(x, tuple) else x for x in enc.debug_log] == c["debug_log"]
        enc = AC(CDFPredictor(c["cdf"]), c["prec"]).to_bin
        enc.debug_log = []                           # falsy: nothing logged
        list(enc.bits(c["syms"]))
        assert enc.debug_log == []


def test_batch_decode_rejects_bad_shapes():
    """BatchCoder.decode / decode_open validate tables, outputs and bit buffers
    instead of letting the kernels read or write out of bounds."""
    from lac_amd.batch import BatchCoder
    dev = "cuda:0"
    V, B = 64, 4
    coder = BatchCoder(V, B, prec=24, device=dev)
    pmf = torch.ones((3, B, V), dtype=torch.int32, device=dev)
    coder.encode(pmf, torch.zeros((3, B), dtype=torch.int32, device=dev))
    coder.finish()
    coder.decode_open()
    with pytest.raises(ValueError):
        coder.decode(torch.ones((3, B - 1, V), dtype=torch.int32, device=dev))
    with pytest.raises(ValueError):
        coder.decode(pmf, out=torch.empty((2, B), dtype=torch.int32, device=dev))
    with pytest.raises(TypeError):
        coder.decode(pmf, out=torch.empty((3, B), dtype=torch.int64, device=dev))
    bits = torch.zeros((B, 16), dtype=torch.uint8, device=dev)
    with pytest.raises(TypeError):
        coder.decode_open(bits.view(torch.int64), torch.zeros(B, dtype=torch.int64, device=dev))
    with pytest.raises(TypeError):
        coder.decode_open(bits, torch.zeros(B, dtype=torch.int32, device=dev))
    with pytest.raises(ValueError):
        coder.decode_open(bits, torch.zeros(B + 1, dtype=torch.int64, device=dev))
    # nbits beyond the row: that stream fails (sticky LAC_E_ARG), the others decode
    nb = torch.tensor([8, 16 * 8, 16 * 8 + 1, 0], dtype=torch.int64, device=dev)
    coder.decode_open(bits, nb)
    out = coder.decode(pmf)
    rc, err, _ = coder.status()
    assert err.tolist() == [0, 0, -1, 0]
    assert (out[:, 2] == -1).all() and (out[:, [0, 1, 3]] >= 0).all()
    coder.close()


def test_fused_decode_many_streams_with_failed_streams():
    """6000 streams through the one-wave-per-stream decoder (more streams than
    resident waves: two dispatch rounds and a partial third), a few of them failed
    at open (sticky LAC_E_ARG from nbits beyond the row): those report -1, every
    other stream decodes, on u32 and u64 rows; the stats path agrees."""
    from lac_amd.batch import BatchCoder
    dev = "cuda:0"
    for bits_w, V in ((32, 2048), (64, 1024)):
        B, T, prec = 6000, 5, 40
        g = torch.Generator(device=dev).manual_seed(bits_w)
        pmf = (torch.randint(1, 1 << 20, (T, B, V), generator=g, device=dev, dtype=torch.int64))
        pmf = pmf.to(torch.int32) if bits_w == 32 else pmf
        sym = torch.randint(0, V, (T, B), generator=g, device=dev, dtype=torch.int32)
        coder = BatchCoder(V, B, prec=prec, pmf_bits=bits_w, capacity_bits=T * (prec + 2) + 256, device=dev)
        coder.encode_job(pmf, sym)
        coder.raise_on_error()
        bits = coder.bits_tensor()
        nb = coder.nbits_tensor()
        bad = torch.arange(0, B, 997, device=dev)                # a few streams on different waves
        nb_bad = nb.clone()
        nb_bad[bad] = bits.shape[1] * 8 + 1
        coder.set_decode_path("fused")
        coder.decode_open(bits, nb_bad)
        out = coder.decode(pmf)
        rc, err, _ = coder.status()
        ok = torch.ones(B, dtype=torch.bool, device=dev)
        ok[bad] = False
        assert (torch.from_numpy(err).to(dev)[bad] == -1).all() and (torch.from_numpy(err).to(dev)[ok] == 0).all()
        assert (out[:, bad] == -1).all() and torch.equal(out[:, ok], sym[:, ok])
        coder.set_decode_path("stats")
        coder.decode_open(bits, nb)
        assert torch.equal(coder.decode(pmf), sym)
        coder.close()


def test_acsampler_per_token_pdfs_bits_and_entropy():
    """ACSampler with a new float pdf per token: GPU bits and bits_per_token ==
    the reference's (tests/golden/acsampler_cb.json); the host Region mirror
    agrees with the GPU coder's registers at flush."""
    from lac_amd.sampler import ACSampler
    for case in load_golden("acsampler_cb.json")["cases"]:
        s = ACSampler(48)
        bits, ent = [], []
        s.compress_tokens = iter(case["tokens"])
        s.compress_output = bits.append
        s.bits_per_token = ent.append
        for pdf in case["pdfs"]:
            s.sample(pdf)
        s.flush_compress()
        assert "".join(map(str, bits)) == case["bits"]
        assert ent == case["entropy"]


def test_synth_tables_one_generator_equal_per_step_generators():
    """synth.softmax_tables / logits_batch reseed one torch.Generator per step: the tables
    and symbols equal the per-step-generator form they replaced (thousands of
    device generators crashed torch.randn under rocprofv3 --pmc)."""
    import torch
    from lac_amd import synth
    dev = "cuda"
    T, B, V, seed = 5, 7, 1000, 99
    for scale, bits in ((31, 32), (60, 64)):
        got, gs = synth.softmax_tables(T, B, V, seed=seed, device=dev, scale_bits=scale, storage_bits=bits)
        for t in range(T):
            g = torch.Generator(device=dev)
            g.manual_seed(seed + t)
            logits = torch.randn((B, V), generator=g, device=dev, dtype=torch.float32) * 3.0
            q = torch.clamp(torch.floor(torch.softmax(logits.double(), dim=-1) * float(1 << scale)),
                            min=2 if scale >= 60 else 1).to(torch.int64)
            cdf = torch.cumsum(q, dim=-1)
            u = torch.rand((B,), generator=g, device=dev, dtype=torch.float64)
            tgt = torch.minimum((u * cdf[:, -1].double()).floor().long(), cdf[:, -1] - 1)
            s = torch.searchsorted(cdf, tgt.unsqueeze(1), right=True).squeeze(1).to(torch.int32)
            assert torch.equal(got[t], q.to(got.dtype)) and torch.equal(gs[t], s), (scale, t)
    lg, _ = synth.logits_batch(T, B, V + 8, seed=seed, device=dev, quantise=lambda x: x.float().to(torch.int64))
    for t in range(T):
        g = torch.Generator(device=dev)
        g.manual_seed(seed + t)
        want = (torch.randn((B, V + 8), generator=g, device=dev, dtype=torch.float32) * 3.0).to(torch.bfloat16)
        assert torch.equal(lg[t], want), t
