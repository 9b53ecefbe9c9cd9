"""The caller-side quantiser pinned to the reference.

tests/golden/llama_cases.json records what the reference's own Llama_AC
(llama_compress.py:14-61) computes when driven by tests/fake_llm.py: per step
the logits, the int64 CDF of calc_dist (:24-30), minp (:43-45) and the sliding
window (:31-39), and the exact-int A_to_bin bits on those CDFs
(tools/gen_golden_llama.py).  lac_amd.llm.Llama_AC must reproduce all of it.
"""
import hashlib

import numpy as np
import pytest

from conftest import load_golden
from fake_llm import FakeLlama, HeadLlama

CASES = load_golden("llama_cases.json")["cases"]
REFUSE = load_golden("llama_cases.json")["refuse"]


def _llm(case):
    if "heads" in case:
        return HeadLlama(case["vocab"], case["n_ctx"], case["heads"], case["floor"])
    return FakeLlama(case["vocab"], case["n_ctx"], case["seed"], scale=case.get("scale", 3.0))


def _sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.mark.parametrize("case", CASES + REFUSE, ids=[c["name"] for c in CASES + REFUSE])
def test_llama_ac_tables_match_reference(case):
    """Logits, int64 CDFs, minp (zeros included: the peaky cases' rows have zero CDF
    steps and minp 0) and window, step by step, equal the reference adapter's."""
    from lac_amd.llm import Llama_AC, quantise_logits
    llm = _llm(case)
    p = Llama_AC(llm)
    for i, (t, want) in enumerate(zip(case["tokens"], case["steps"])):
        logits = np.asarray(llm._scores[-1], dtype=np.float32)
        assert _sha(logits.tobytes()) == want["logits_sha256"], i
        cdf = p.dist
        assert _sha(np.asarray(cdf, dtype="<i8").tobytes()) == want["cdf_sha256"], i
        assert _sha(np.asarray(quantise_logits(logits), dtype="<i8").tobytes()) == want["cdf_sha256"], i
        assert p.minp == want["minp"] and len(p.past) == want["window"], i
        if "cdf" in want:
            assert [int(x) for x in cdf] == want["cdf"], i
        p.accept(t)
    assert max(s["window"] for s in case["steps"]) == min(case["n_ctx"] - 1, len(case["tokens"]))


def test_peaky_cases_have_zero_steps():
    """The fixture covers the reference's always-fudged branch: rows whose float64
    cumsum absorbed entries (zero CDF steps), so Llama_AC.minp == 0 and
    fudged_dist fudges at every width (arith_code.py:84)."""
    peaky = [c for c in CASES if c.get("scale", 3.0) >= 12]
    assert len(peaky) == 2 and {c["vocab"] for c in peaky} == {1000, 32000}
    for c in peaky:
        assert c["zero_step_rows"] == len(c["tokens"]) and all(s["minp"] == 0 for s in c["steps"])


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_fudge_decisions_agree_on_reference_rows(case):
    """Every recorded row's declared minp (the reference's) and its smallest positive
    entry give the same fudge decision at every width: the build codes them."""
    from lac_amd.coder import fudge_decisions_agree
    from lac_amd.llm import Llama_AC
    p = Llama_AC(_llm(case))
    for t, want in zip(case["tokens"], case["steps"]):
        r = p.pmf_row()
        assert p.minp == want["minp"]
        assert fudge_decisions_agree(int(r.sum(dtype=object)), p.minp, int(r[r > 0].min()), case["prec"])
        p.accept(t)


@pytest.mark.parametrize("case", REFUSE, ids=[c["name"] for c in REFUSE])
def test_refusal_rows(case):
    """Rows with zero steps whose every positive entry is >= 2^12 (HeadLlama): the
    reference (minp 0) fudges at every width, the table's smallest positive entry
    would not at the widest -- the build refuses the first such row rather than code
    it differently (lac_amd.coder.fudge_decisions_agree)."""
    from lac_amd.coder import fudge_decisions_agree
    from lac_amd.llm import Llama_AC
    p = Llama_AC(_llm(case))
    k = case["refuse_at_step"]
    for i, t in enumerate(case["tokens"][:k + 1]):
        r = p.pmf_row()
        assert int(r[r > 0].min()) == case["min_positive"][i] >= 1 << 12
        agree = fudge_decisions_agree(int(r.sum(dtype=object)), p.minp, int(r[r > 0].min()), case["prec"])
        assert agree == (i != k), i
        p.accept(t)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_exact_bits_on_reference_tables(case):
    """The oracle, on the CDFs this adapter yields, gives the reference's exact-int bits
    (on the peaky cases the oracle's minp is the smallest positive entry, which fudges
    wherever the reference's minp 0 does: the test above)."""
    from lac_amd.llm import Llama_AC
    from oracle import restate
    p = Llama_AC(_llm(case))
    rows = []
    for t in case["tokens"]:
        rows.append([int(x) for x in p.pmf_row()])
        p.accept(t)
    data, L = restate.encode_bytes(rows, case["tokens"], case["prec"])
    assert L == case["exact_L"] and data.hex() == case["exact_bytes"]


def test_tiny_lm_cached_steps_match_forward():
    """TinyCausalLM's key/value-cache steps (what LogitsCompressor and TorchLLM run,
    O(1) model work per token) compute the teacher-forced forward's logits, and
    TorchLLM's incremental eval matches re-running the window -- across the
    sliding-window rebuild past n_ctx (CPU, float32)."""
    torch = pytest.importorskip("torch")
    from lac_amd.llm import TinyCausalLM, TorchLLM
    m = TinyCausalLM(vocab=300, d=32, layers=2, heads=2, max_len=64, seed=3).eval()
    x = torch.from_numpy(np.random.default_rng(1).integers(0, 300, (3, 20)))
    with torch.no_grad():
        full = m(x)
        cache = m.init_cache(3, 20)
        steps = torch.stack([m.step(x[:, t], cache, t) for t in range(20)], 1)
    assert torch.allclose(full, steps, atol=1e-4, rtol=1e-4)

    class Plain(torch.nn.Module):                              # forward() only: the window re-run
        def forward(self, z):
            return m(z)
    inc, win = TorchLLM(m, n_ctx=12, device="cpu"), TorchLLM(Plain(), n_ctx=12, device="cpu")
    assert inc.incremental and not win.incremental
    for t in range(1, 30):
        inc.eval([t])
        win.eval([t])
        assert np.allclose(inc._scores, win._scores, atol=1e-4), t
    assert len(inc.tokens) == 12                                # trimmed to the window past n_ctx
    before = inc._scores.copy()
    inc.eval([])                                               # nothing new: the last logits stand
    assert np.array_equal(inc._scores, before)
    inc.reset()
    with pytest.raises(ValueError):
        inc.eval([])
    inc.eval([1, 2, 3])
    win.reset()
    win.eval([1, 2, 3])
    assert np.allclose(inc._scores, win._scores, atol=1e-4)
    inc.eval([])
    assert np.allclose(inc._scores, win._scores, atol=1e-4)
