#!/usr/bin/env python3
"""The coder's cost per position inside a ROCm serving loop (SURVEY
§8(f)3): llama_compress.py:31-39 feeds one token per model step, and the decoder needs
position t's symbol before the model can run step t+1, so the coder sits between two
model steps at every position.

    python tools/serving_bench.py --streams 1 --positions 256 [--model tiny|small] [--out F]

Per position t, ``LogitsCompressor.decompress`` (lac_amd/llm.py) runs one cached model
step (TinyCausalLM, random init: no checkpoint can be fetched) to bf16 logits [1, B,
V=32000] in HBM, then ``BatchCoder.decode_logits`` -- k_q1_stats (row statistics of the
q1 tables, computed in-kernel) + k_q1_decode (the per-stream chain) -- whose symbols feed
the next step on the device (no host round trip).  Reported, in microseconds per
position (wall clock over the whole loop, one synchronisation at its end, after a warm
run of the same loop):

* ``decompress``: the serving loop itself (model + coder, as a user runs it);
* ``model_only``: the same loop with the tokens known and no coder;
* ``coder_only``: decode_logits over the same logits, resident in HBM, position by
  position (launches included);
* ``coder_device``: the coder's kernels' device time per position (hipEvents of liblac
  on the coder's stream, lac_profile_*), split into k_q1_stats and k_q1_decode;
* the same three for compress (encode_logits per position);
* ``coder_share`` = coder_only / decompress.

Bits are checked: decompress returns the tokens compress coded.  Prints one JSON line.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

MODELS = {"tiny": dict(d=64, layers=2, heads=4), "small": dict(d=512, layers=4, heads=8)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=1)
    ap.add_argument("--positions", type=int, default=256)
    ap.add_argument("--vocab", type=int, default=32000)
    ap.add_argument("--model", choices=sorted(MODELS), default="tiny")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    from lac_amd.llm import LogitsCompressor, TinyCausalLM
    dev = torch.device("cuda", 0)
    B, T, V = a.streams, a.positions, a.vocab
    cfg = MODELS[a.model]
    model = TinyCausalLM(vocab=V, max_len=max(T, 16), seed=7, **cfg).to(dev).eval()
    lc = LogitsCompressor(model, V, prec=48, logits_dtype=torch.bfloat16, device=dev)
    g = torch.Generator(device=dev).manual_seed(11)
    tokens = torch.randint(0, V, (B, T), generator=g, device=dev)
    sync = torch.cuda.synchronize

    def timed(fn, reps=2):
        best = None
        for _ in range(reps):                              # the first run warms kernels and clocks
            sync()
            t0 = time.perf_counter()
            r = fn()
            sync()
            dt = time.perf_counter() - t0
            best = dt if best is None or dt < best else best
        return best, r

    # ---- the serving loops (model + coder)
    t_comp, (data, nbits) = timed(lambda: lc.compress(tokens))
    t_dec, got = timed(lambda: lc.decompress(data, nbits, T))
    ok = bool(torch.equal(got.cpu(), tokens.cpu()))

    # ---- the model alone: the same cached steps, tokens known
    def model_only():
        last = None
        for _, lg in lc._steps(B, T, lambda t: tokens[:, t]):
            last = lg
        return last
    t_model, _ = timed(model_only)

    # ---- the coder alone over resident logits, position by position
    logits = [lg.clone() for _, lg in lc._steps(B, T, lambda t: tokens[:, t])]
    sym = tokens.t().contiguous().to(torch.int32)
    coder = lc._coder(B, T)
    buf_stride = max(8, (max(len(d) for d in data) + 8) // 8 * 8)
    import numpy as np
    host = np.zeros((B, buf_stride), dtype=np.uint8)
    for b, d in enumerate(data):
        host[b, :len(d)] = np.frombuffer(d, dtype=np.uint8)
    dbits = torch.from_numpy(host).to(dev)
    dnb = torch.as_tensor(np.asarray(nbits, dtype=np.int64), device=dev)
    out = torch.empty((T, B), dtype=torch.int32, device=dev)

    def coder_decode():
        coder.decode_open(dbits, dnb)
        for t in range(T):
            coder.decode_logits(logits[t], out=out[t:t + 1])
        return out

    def coder_encode():
        coder.reset()
        for t in range(T):
            coder.encode_logits(logits[t], sym[t:t + 1])
        coder.finish()
    t_cdec, _ = timed(coder_decode)
    dec_ok = bool(torch.equal(out, sym))
    t_cenc, _ = timed(coder_encode)
    enc_bytes, enc_nb = coder.to_bytes()
    enc_ok = all(enc_bytes[b] == data[b] for b in range(B))

    # ---- device time of the coder's kernels (liblac's hipEvents on its stream)
    def device_ms(fn):
        ms = (C.c_double * 8)()
        cnt = (C.c_int64 * 8)()
        coder.lib.lac_profile_read(coder.ctx, None, None, 1)
        coder.lib.lac_profile_enable(coder.ctx, 1)
        fn()
        sync()
        coder.lib.lac_profile_enable(coder.ctx, 0)
        coder.lib.lac_profile_read(coder.ctx, C.cast(ms, C.c_void_p), C.cast(cnt, C.c_void_p), 1)
        return {k: (ms[i] * 1e3 / T, int(cnt[i])) for k, i in
                (("row_stats", 0), ("encode", 1), ("finish", 2), ("q1_stats", 6), ("q1_decode", 7)) if cnt[i]}
    ddec = device_ms(coder_decode)
    denc = device_ms(coder_encode)
    coder.close()

    us = lambda s: 1e6 * s / T                               # noqa: E731
    res = {
        "what": "coder cost per position in the ROCm serving loop (LogitsCompressor, bf16 logits)",
        "model": f"TinyCausalLM {cfg} (random init), cached step per position",
        "vocab": V, "streams": B, "positions": T, "prec": 48,
        "roundtrip_ok": ok and dec_ok and enc_ok,
        "decompress_us_per_pos": us(t_dec), "compress_us_per_pos": us(t_comp),
        "model_only_us_per_pos": us(t_model),
        "coder_decode_only_us_per_pos": us(t_cdec), "coder_encode_only_us_per_pos": us(t_cenc),
        "coder_decode_device_us_per_pos": {k: round(v[0], 3) for k, v in ddec.items()},
        "coder_encode_device_us_per_pos": {k: round(v[0], 3) for k, v in denc.items()},
        "coder_share_of_decompress": t_cdec / t_dec,
        "coder_share_of_compress": t_cenc / t_comp,
        "logits_bytes_per_pos": B * lc.vcode * 2,
    }
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            f.write(line + "\n")
    return 0 if res["roundtrip_ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
