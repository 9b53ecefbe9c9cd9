"""LLM predictors for the GPU coder: the ``Llama_AC`` adapter and a ROCm torch backend.

``Llama_AC`` keeps the surface of /root/reference/llama_compress.py:14-61:
``reset`` primes the model with BOS (=1), ``accept`` evaluates the accepted token
and, when the context is full, keeps the last ``n_ctx // overlap`` tokens and
re-evaluates them; ``calc_dist`` turns the last logits into an integer CDF
(``max(2, p * 2^60)``, float64, :24-30).  Any object with llama_cpp.Llama's
duck type works as ``llm``: ``reset()``, ``eval(tokens)``, ``n_ctx()`` and
``_scores`` (2-D, last row = next-token logits).

``TorchLLM`` provides that duck type for a PyTorch causal LM on the GPU, so a
ROCm model drops in where llama.cpp was: one cached step per evaluated token
for a module with a key/value cache (TinyCausalLM), else the window re-run on
every ``eval`` -- the same op sequence on the encode and the decode side either
way, which is what makes the quantised tables, and the bitstream, reproducible.

Coding goes through lac_amd.coder (GPU); this module only produces tables.
"""
from __future__ import annotations

import numpy as np

from .coder import ProbPredictor


def quantise_logits(logits) -> np.ndarray:
    """logits -> inclusive int64 CDF, the reference's quantiser (llama_compress.py:24-30),
    the same numpy operations in the same order and dtypes: exp and normalise in the
    logits' own dtype (float32 for llama.cpp's scores), scale by the Python int
    2^60 (a weak scalar: the product keeps that dtype), widen to float64, clip at 2,
    float64 running sum, truncate to int64.  Pinned to the reference by
    tests/golden/llama_cases.json (tests/test_llama_host.py)."""
    pdf = np.exp(logits)
    pdf /= np.sum(pdf)
    return np.cumsum(np.clip((pdf * (1 << 60)).astype(float), 2, None)).astype(np.int64)


class Llama_AC(ProbPredictor):
    """Model-driven predictor (llama_compress.py:14-61) for lac_amd.coder.AC."""

    def __init__(self, llm, maxtoks=2048):
        super().__init__(0)
        self.llm = llm
        self.overlap = 2
        self.reset()

    def reset(self):
        self.past = [1]
        self.llm.reset()
        self.llm.eval([1])

    def calc_dist(self):
        self.dcache = quantise_logits(self.llm._scores[-1])
        return self.dcache

    def pmf_row(self):
        """The current table as a uint64 pmf row (what the coder uploads)."""
        cdf = self.dist
        pmf = np.empty(len(cdf), dtype=np.uint64)
        pmf[0] = cdf[0]
        pmf[1:] = np.diff(cdf).astype(np.uint64)
        return pmf

    def accept(self, symbol):
        self.past.append(symbol)
        n_ctx = self.llm.n_ctx()
        if len(self.past) == n_ctx:
            self.past = self.past[n_ctx - n_ctx // self.overlap:]
            self.llm.reset()
            self.llm.eval(self.past)
        else:
            self.llm.eval([symbol])
        return super().accept(symbol)

    def copy(self):
        return Llama_AC(self.llm)

    @property
    def minp(self):
        return int(min(self.dist[0], np.min(np.diff(self.dist))))


class TorchLLM:
    """llama_cpp.Llama's duck type over a torch causal LM on a HIP device.

    A module with ``init_cache(B, T)`` / ``step(tokens[B], cache, t)`` (as
    TinyCausalLM) is run incrementally: each evaluated token is one step against
    a key/value cache, so a sequence costs O(T) steps as with llama.cpp's own KV
    cache.  Past ``n_ctx`` tokens the window slides with every token, so each
    eval is one forward over the window and the history is trimmed to it
    (Llama_AC resets before that happens).  ``eval([])`` keeps the last logits.
    Any other module
    (``module(tokens[1, t]) -> logits[1, t, V]``) re-runs the window on every
    ``eval``.  Either way the encode and decode sides issue the same sequence of
    calls, which is what makes the logits -- and the tables and bitstream --
    reproducible."""

    def __init__(self, module, n_ctx=512, device="cuda"):
        import torch
        self.module = module.to(device).eval()
        self.device = torch.device(device)
        self._n_ctx = n_ctx
        self.incremental = hasattr(module, "step") and hasattr(module, "init_cache")
        self.reset()

    def n_ctx(self):
        return self._n_ctx

    def reset(self):
        self.tokens = []
        self._scores = None
        self._cache = None
        self._pos = 0

    def eval(self, tokens):
        import torch
        new = [int(t) for t in tokens]
        if not new:
            if self._scores is None:
                raise ValueError("eval([]) before any token: there are no logits yet")
            return                                          # nothing new: the last logits stand
        self.tokens.extend(new)
        with torch.no_grad():
            if self.incremental and len(self.tokens) <= self._n_ctx:
                if self._cache is None:                     # fresh (or after a slide): replay the window
                    self._cache = self.module.init_cache(1, self._n_ctx)
                    self._pos = 0
                    new = self.tokens
                for t in new:
                    x = torch.tensor([t], dtype=torch.long, device=self.device)
                    logits = self.module.step(x, self._cache, self._pos)[0].float()
                    self._pos += 1
            else:
                # past n_ctx the window slides every token, so its positions shift and a
                # cache cannot be reused: one forward over the window, the history
                # trimmed to it (tokens before it can no longer matter)
                window = self.tokens[-self._n_ctx:]
                self.tokens = list(window)
                self._cache = None
                x = torch.tensor([window], dtype=torch.long, device=self.device)
                logits = self.module(x)[0, -1].float()
        self._scores = logits.cpu().numpy()[None, :]


class TinyCausalLM:
    """A small random-init GPT-style causal transformer (torch) for tests and demos
    -- a stand-in for a real checkpoint, which cannot be fetched offline.  Pre-LN
    blocks (attention + 4d MLP); ``forward(tokens[B, T]) -> logits[B, T, V]``
    teacher-forced, and ``init_cache`` / ``step`` for incremental decoding with a
    key/value cache: every step has the same shapes (the cache is T long and
    masked past position t), so a step runs the same kernels whoever calls it."""

    def __new__(cls, vocab=32000, d=64, layers=2, heads=4, max_len=512, seed=0):
        import math

        import torch
        import torch.nn as nn

        class _Block(nn.Module):
            def __init__(self):
                super().__init__()
                self.ln1, self.ln2 = nn.LayerNorm(d), nn.LayerNorm(d)
                self.qkv, self.proj = nn.Linear(d, 3 * d), nn.Linear(d, d)
                self.fc1, self.fc2 = nn.Linear(d, 4 * d), nn.Linear(4 * d, d)

            def _heads(self, z):                                  # [B, t, d] -> [B, H, t, dh]
                return z.view(z.shape[0], z.shape[1], heads, d // heads).transpose(1, 2)

            def attend(self, q, k, v, mask):
                a = torch.softmax((q @ k.transpose(-1, -2)) / math.sqrt(d // heads) + mask, dim=-1) @ v
                return a.transpose(1, 2).reshape(q.shape[0], q.shape[2], d)

            def mlp(self, h):
                return h + self.fc2(torch.nn.functional.gelu(self.fc1(self.ln2(h))))

            def forward(self, h, mask):
                q, k, v = (self._heads(z) for z in self.qkv(self.ln1(h)).split(d, dim=-1))
                return self.mlp(h + self.proj(self.attend(q, k, v, mask)))

            def step(self, h, kv, t, mask):                      # h [B, 1, d]; kv: this block's (K, V) [B, H, T, dh]
                q, k, v = (self._heads(z) for z in self.qkv(self.ln1(h)).split(d, dim=-1))
                kv[0][:, :, t:t + 1] = k
                kv[1][:, :, t:t + 1] = v
                return self.mlp(h + self.proj(self.attend(q, kv[0], kv[1], mask)))

        class _M(nn.Module):
            def __init__(self):
                super().__init__()
                g = torch.Generator().manual_seed(seed)
                self.emb = nn.Embedding(vocab, d)
                self.pos = nn.Embedding(max_len, d)
                self.blocks = nn.ModuleList(_Block() for _ in range(layers))
                self.ln = nn.LayerNorm(d)
                self.head = nn.Linear(d, vocab)
                with torch.no_grad():
                    for name, p in self.named_parameters():
                        if ".ln" in name or name.startswith("ln"):
                            continue                              # LayerNorm: weight 1, bias 0
                        p.copy_(torch.randn(p.shape, generator=g) * 0.5)

            def forward(self, x):
                t = x.shape[1]
                mask = torch.triu(torch.full((t, t), float("-inf"), device=x.device), 1)
                h = self.emb(x) + self.pos(torch.arange(t, device=x.device))[None]
                for blk in self.blocks:
                    h = blk(h, mask)
                return self.head(self.ln(h))

            def init_cache(self, B, T):
                p = self.head.weight
                return [(p.new_zeros((B, heads, T, d // heads)), p.new_zeros((B, heads, T, d // heads)))
                        for _ in self.blocks]

            def step(self, tok, cache, t):
                """Logits [B, V] of the next token after tok[B] at position t."""
                T = cache[0][0].shape[2]
                mask = torch.full((T,), float("-inf"), device=tok.device)
                mask[:t + 1] = 0
                h = self.emb(tok[:, None]) + self.pos.weight[t][None, None]
                for blk, kv in zip(self.blocks, cache):
                    h = blk.step(h, kv, t, mask)
                return self.head(self.ln(h))[:, 0]

        return _M()


class LogitsCompressor:
    """Batched LLM compression on the GPU through the logits path (SURVEY §8(f) 1 + 3).

    Step t codes token t with the model's logits after ``[BOS] + tokens[:, :t]``
    (llama_compress.py primes with BOS = 1, :20-23), handed -- cast to
    ``logits_dtype``, in HBM -- straight to the coder's logits entry points: the q1
    tables are computed in-kernel and no pmf is ever written.  Decoding must see
    bit-identical logits, so both sides produce them the same way:

    * incremental (a module with ``init_cache`` / ``step``, e.g. TinyCausalLM):
      one cached step per position on both sides (``encode_logits`` /
      ``decode_logits`` per step) -- O(T) steps each way, as a serving loop;
    * otherwise (``module(tokens[B, T]) -> logits[B, T, V]`` only): compress runs
      one teacher-forced forward, and decompress re-runs the *same* fixed-shape
      [B, T] forward (not-yet-decoded positions 0) before each step -- under the
      causal mask position t never depends on later ones, and equal shapes select
      the same kernels.  O(T) full forwards: for modules without a cache.
    """

    def __init__(self, module, vocab, prec=48, bos=1, logits_dtype=None, device="cuda"):
        import torch
        from .batch import logits_row_multiple
        self.module = module.to(device).eval()
        self.vocab, self.prec, self.bos = int(vocab), int(prec), int(bos)
        self.dtype = logits_dtype or torch.bfloat16
        self.device = torch.device(device)
        self.incremental = hasattr(module, "step") and hasattr(module, "init_cache")
        # the logits kernels read rows as 16-B vectors: a vocab that is not a multiple
        # of 8 (bf16) / 4 (f32) -- GPT-2's 50257, say -- is coded over rows padded
        # with -inf (pad entries get the q1 minimum weight, 1 unit; compress and
        # decompress pad alike, so the code stays lossless)
        m = logits_row_multiple(self.dtype)
        self.vcode = (self.vocab + m - 1) // m * m

    def _fit(self, lg):
        if self.vcode != lg.shape[-1]:
            lg = __import__("torch").nn.functional.pad(lg, (0, self.vcode - lg.shape[-1]), value=float("-inf"))
        return lg.contiguous()

    def _logits(self, ctx):
        import torch
        with torch.no_grad():
            return self._fit(self.module(ctx).to(self.dtype))

    def _steps(self, B, T, feed):
        """Incremental: yields (t, logits [1, B, vcode]) for t < T; feed(t) -> the tokens [B]
        at position t + 1's input (the coded / decoded token t)."""
        import torch
        cache = self.module.init_cache(B, T)
        tok = torch.full((B,), self.bos, dtype=torch.long, device=self.device)
        for t in range(T):
            with torch.no_grad():
                lg = self._fit(self.module.step(tok, cache, t).to(self.dtype))[None]
            yield t, lg
            tok = feed(t)

    def logits(self, tokens):
        """The [B, T, vcode] logits compress codes tokens[B, T] with (for checking)."""
        import torch
        tokens = tokens.to(self.device, torch.long)
        B, T = tokens.shape
        if not self.incremental:
            ctx = torch.cat([torch.full((B, 1), self.bos, dtype=torch.long, device=self.device), tokens[:, :-1]], 1)
            return self._logits(ctx)
        return torch.cat([lg for _, lg in self._steps(B, T, lambda t: tokens[:, t])], 0).transpose(0, 1)

    def _coder(self, B, T):
        from .batch import BatchCoder
        return BatchCoder(self.vcode, B, prec=self.prec, pmf_bits=32, capacity_bits=T * (self.prec + 2) + 256,
                          device=self.device)

    def compress(self, tokens):
        """tokens: int tensor [B, T] -> (list of B byte strings, nbits uint64[B])."""
        import torch
        tokens = tokens.to(self.device, torch.long)
        B, T = tokens.shape
        coder = self._coder(B, T)
        if self.incremental:
            sym = tokens.t().contiguous().to(torch.int32)          # [T, B]
            coder.reset()
            for t, lg in self._steps(B, T, lambda t: tokens[:, t]):
                coder.encode_logits(lg, sym[t:t + 1])
            coder.finish()
        else:
            coder.encode_logits_job(self.logits(tokens).transpose(0, 1), tokens.t().contiguous().to(torch.int32))
        out = coder.to_bytes()
        coder.close()
        return out

    def decompress(self, data, nbits, T):
        """Inverse of compress: B byte strings + bit counts -> tokens [B, T] (long)."""
        import torch
        B = len(data)
        stride = max(8, (max((len(d) for d in data), default=0) + 8) // 8 * 8)
        buf = np.zeros((B, stride), dtype=np.uint8)
        for b, d in enumerate(data):
            buf[b, :len(d)] = np.frombuffer(d, dtype=np.uint8)
        coder = self._coder(B, T)
        bits = torch.from_numpy(buf).to(self.device)
        nb = torch.as_tensor(np.asarray(nbits, dtype=np.int64), device=self.device)
        coder.decode_open(bits, nb)
        out = torch.empty((B, T), dtype=torch.long, device=self.device)
        if self.incremental:
            for t, lg in self._steps(B, T, lambda t: out[:, t]):
                out[:, t] = coder.decode_logits(lg)[0].to(torch.long)
        else:
            ctx = torch.zeros((B, T), dtype=torch.long, device=self.device)
            ctx[:, 0] = self.bos
            for t in range(T):
                lg = self._logits(ctx)[:, t:t + 1, :]            # [B, 1, V]
                s = coder.decode_logits(lg.transpose(0, 1))[0].to(torch.long)
                out[:, t] = s
                if t + 1 < T:
                    ctx[:, t + 1] = s
        coder.raise_on_error()
        coder.close()
        return out
