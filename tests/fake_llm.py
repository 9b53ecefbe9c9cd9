"""A duck-typed stand-in for llama_cpp.Llama: reset(),
eval(tokens), n_ctx() and _scores, whose last row -- the next-token logits --
is a seeded float32 function of the context window.  Used to drive the
reference's Llama_AC (tools/gen_golden_llama.py) and this build's
lac_amd.llm.Llama_AC (tests) with identical logits.  ``scale`` >= 12 makes the
logits peaky enough that the reference's float64 cumsum near 2^60 absorbs the
small entries (zero CDF steps, Llama_AC.minp == 0).  ``HeadLlama`` scripts rows
with a few dominant logits over a flat floor (a quantised row whose every positive
entry is >= 2^12)."""
import numpy as np


class FakeLlama:
    def __init__(self, vocab, n_ctx, seed, scale=3.0):
        self.vocab, self._n_ctx, self.seed, self.scale = vocab, n_ctx, seed, scale
        self.toks = []
        self._scores = None

    def n_ctx(self):
        return self._n_ctx

    def reset(self):
        self.toks = []
        self._scores = None

    def eval(self, tokens):
        self.toks.extend(int(t) for t in tokens)
        h = self.seed
        for t in self.toks[-self._n_ctx:]:
            h = (h * 1000003 + t + 1) % (1 << 61)
        logits = (np.random.default_rng(h).standard_normal(self.vocab) * self.scale).astype(np.float32)
        self._scores = logits[None, :]


class HeadLlama(FakeLlama):
    """Rows of ``floor`` everywhere except the first entries, which take ``head``
    (one list of head values per row, rows taken in turn by the number of tokens
    evaluated since the last reset)."""

    def __init__(self, vocab, n_ctx, heads, floor=10.0):
        super().__init__(vocab, n_ctx, 0)
        self.heads, self.floor = [list(h) for h in heads], float(floor)

    def eval(self, tokens):
        self.toks.extend(int(t) for t in tokens)
        h = self.heads[(len(self.toks) - 1) % len(self.heads)]
        logits = np.full(self.vocab, self.floor, dtype=np.float32)
        logits[:len(h)] = np.asarray(h, dtype=np.float32)
        self._scores = logits[None, :]
