"""LLM predictors for the GPU coder: the ``Llama_AC`` adapter and a ROCm torch backend.

``Llama_AC`` keeps the surface of /root/reference/llama_compress.py:14-61:
``reset`` primes the model with BOS (=1), ``accept`` evaluates the accepted token
and, when the context is full, keeps the last ``n_ctx // overlap`` tokens and
re-evaluates them; ``calc_dist`` turns the last logits into an integer CDF
(``max(2, p * 2^60)``, float64, :24-30).  Any object with llama_cpp.Llama's
duck type works as ``llm``: ``reset()``, ``eval(tokens)``, ``n_ctx()`` and
``_scores`` (2-D, last row = next-token logits).

``TorchLLM`` provides that duck type for a PyTorch causal LM on the GPU
(``module(tokens[1, t]) -> logits[1, t, V]``), so a ROCm model drops in where
llama.cpp was.  It re-runs the window on every ``eval`` -- the same op sequence
on the encode and the decode side, which is what makes the quantised tables,
and therefore the bitstream, reproducible.

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
    """llama_cpp.Llama's duck type over a torch causal LM on a HIP device."""

    def __init__(self, module, n_ctx=512, device="cuda"):
        import torch
        self.module = module.to(device).eval()
        self.device = torch.device(device)
        self._n_ctx = n_ctx
        self.tokens = []
        self._scores = None

    def n_ctx(self):
        return self._n_ctx

    def reset(self):
        self.tokens = []
        self._scores = None

    def eval(self, tokens):
        import torch
        self.tokens.extend(int(t) for t in tokens)
        window = self.tokens[-self._n_ctx:]
        with torch.no_grad():
            x = torch.tensor([window], dtype=torch.long, device=self.device)
            logits = self.module(x)[0, -1].float()
        self._scores = logits.cpu().numpy()[None, :]


class TinyCausalLM:
    """A small random-init causal transformer (torch) for tests and demos -- a
    stand-in for a real checkpoint, which cannot be fetched offline."""

    def __new__(cls, vocab=32000, d=64, layers=2, heads=4, max_len=512, seed=0):
        import torch
        import torch.nn as nn

        class _M(nn.Module):
            def __init__(self):
                super().__init__()
                g = torch.Generator().manual_seed(seed)
                self.emb = nn.Embedding(vocab, d)
                self.pos = nn.Embedding(max_len, d)
                layer = nn.TransformerEncoderLayer(d, heads, 4 * d, dropout=0.0, batch_first=True)
                self.body = nn.TransformerEncoder(layer, layers)
                self.head = nn.Linear(d, vocab)
                with torch.no_grad():
                    for p in self.parameters():
                        p.copy_(torch.randn(p.shape, generator=g) * 0.5)

            def forward(self, x):
                t = x.shape[1]
                mask = torch.triu(torch.full((t, t), float("-inf"), device=x.device), 1)
                h = self.emb(x) + self.pos(torch.arange(t, device=x.device))[None]
                return self.head(self.body(h, mask=mask, is_causal=True))

        return _M()


class LogitsCompressor:
    """Batched LLM compression on the GPU through the logits path (SURVEY §8(f) 1 + 3).

    ``compress(tokens[B, T])`` runs the causal LM once, teacher-forced on
    ``[BOS] + tokens[:, :-1]`` (llama_compress.py primes with BOS = 1, :20-23),
    and hands its logits -- cast to ``logits_dtype``, still [B, T, V] in HBM --
    straight to ``BatchCoder.encode_logits_job`` as a strided [T, B, V] view: the
    q1 tables are computed in-kernel and no pmf is ever written.

    ``decompress`` must see bit-identical logits.  It re-runs the *same*
    fixed-shape forward ([B, T], not-yet-decoded positions filled with 0) before
    each step: under the causal mask position t never depends on later positions,
    and equal shapes select the same kernels, so row t is computed by the
    identical op sequence as in ``compress``.  (An incremental KV-cache decode
    would change shapes and kernels, and with them the low bits of the logits.)
    O(T) forwards: a demonstration driver, not a serving loop.
    """

    def __init__(self, module, vocab, prec=48, bos=1, logits_dtype=None, device="cuda"):
        import torch
        from .batch import logits_row_multiple
        self.module = module.to(device).eval()
        self.vocab, self.prec, self.bos = int(vocab), int(prec), int(bos)
        self.dtype = logits_dtype or torch.bfloat16
        self.device = torch.device(device)
        # the logits kernels read rows as 16-B vectors: a vocab that is not a multiple
        # of 8 (bf16) / 4 (f32) -- GPT-2's 50257, say -- is coded over rows padded
        # with -inf (pad entries get the q1 minimum weight, 1 unit; compress and
        # decompress pad alike, so the code stays lossless)
        m = logits_row_multiple(self.dtype)
        self.vcode = (self.vocab + m - 1) // m * m

    def _logits(self, ctx):
        import torch
        with torch.no_grad():
            lg = self.module(ctx).to(self.dtype)
            if self.vcode != lg.shape[-1]:
                lg = torch.nn.functional.pad(lg, (0, self.vcode - lg.shape[-1]), value=float("-inf"))
            return lg.contiguous()

    def _coder(self, B, T):
        from .batch import BatchCoder
        return BatchCoder(self.vcode, B, prec=self.prec, pmf_bits=32, capacity_bits=T * (self.prec + 2) + 256,
                          device=self.device)

    def compress(self, tokens):
        """tokens: int tensor [B, T] -> (list of B byte strings, nbits uint64[B])."""
        import torch
        tokens = tokens.to(self.device, torch.long)
        B, T = tokens.shape
        ctx = torch.cat([torch.full((B, 1), self.bos, dtype=torch.long, device=self.device), tokens[:, :-1]], 1)
        lg = self._logits(ctx)                                   # [B, T, V]
        coder = self._coder(B, T)
        coder.encode_logits_job(lg.transpose(0, 1), tokens.t().contiguous().to(torch.int32))
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
        ctx = torch.zeros((B, T), dtype=torch.long, device=self.device)
        ctx[:, 0] = self.bos
        out = torch.empty((B, T), dtype=torch.long, device=self.device)
        for t in range(T):
            lg = self._logits(ctx)[:, t:t + 1, :]                # [B, 1, V]
            s = coder.decode_logits(lg.transpose(0, 1))[0].to(torch.long)
            out[:, t] = s
            if t + 1 < T:
                ctx[:, t + 1] = s
        coder.raise_on_error()
        coder.close()
        return out
