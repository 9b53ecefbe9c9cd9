#!/usr/bin/env python3
"""Decode-kernel timing on the bench workload (tuning aid, not the metric).

    python tools/dec_bench.py [--pmf-bits 64] [--vocab 32000] [--streams 4096]
                              [--tokens 16] [--reps 5] [--input pmf|logits-bf16|logits-f32]

Encodes one job, then decodes it --reps times; reports the decode kernels'
device time (liblac.so's hipEvents) per step and the achieved GB/s of
algorithmic bytes (B x (V x e + 4) per step), plus a round-trip check.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--vocab", type=int, default=32000)
    ap.add_argument("--streams", type=int, default=4096)
    ap.add_argument("--tokens", type=int, default=16)
    ap.add_argument("--prec", type=int, default=48)
    ap.add_argument("--pmf-bits", type=int, default=32)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--input", default="pmf")
    ap.add_argument("--decode-path", default="auto")
    a = ap.parse_args()
    import torch
    from lac_amd import synth
    from lac_amd.batch import BatchCoder
    dev = torch.device("cuda", 0)
    V, B, T, P = a.vocab, a.streams, a.tokens, a.prec
    logits_in = a.input != "pmf"
    coder = BatchCoder(V, B, prec=P, pmf_bits=a.pmf_bits, capacity_bits=T * (P + 2) + 256, device=dev)
    if logits_in:
        e = 2 if a.input == "logits-bf16" else 4
        tab, sym = synth.logits_batch(T, B, V, device=dev, dtype=torch.bfloat16 if e == 2 else torch.float32,
                                      quantise=coder.quantize_logits)
        coder.encode_logits_job(tab, sym)
        dec = coder.decode_logits
    else:
        e = a.pmf_bits // 8
        tab, sym = synth.softmax_tables(T, B, V, device=dev, scale_bits=31 if a.pmf_bits == 32 else 60)
        coder.encode_job(tab, sym)
        dec = coder.decode
    if a.decode_path != "auto":
        coder.set_decode_path(a.decode_path)
    coder.raise_on_error()
    coder.decode_open()
    out = dec(tab)
    torch.cuda.synchronize()
    ok = bool(torch.equal(out, sym))
    ms = (C.c_double * 8)()
    cnt = (C.c_int64 * 8)()
    coder.lib.lac_profile_read(coder.ctx, None, None, 1)
    coder.lib.lac_profile_enable(coder.ctx, 1)
    for _ in range(a.reps):
        coder.decode_open()
        out = dec(tab)
    torch.cuda.synchronize()
    coder.lib.lac_profile_enable(coder.ctx, 0)
    coder.lib.lac_profile_read(coder.ctx, C.cast(ms, C.c_void_p), C.cast(cnt, C.c_void_p), 1)
    ok = ok and bool(torch.equal(out, sym))
    kids = [k for k in (3, 5, 6, 7) if cnt[k]]
    step_ms = sum(ms[k] for k in kids) / (a.reps * T)
    print(json.dumps({"vocab": V, "streams": B, "tokens": T, "elem_bytes": e, "input": a.input,
                      "per_kernel_ms_per_step": {k: ms[k] / (a.reps * T) for k in kids},
                      "ms_per_step": step_ms, "sym_per_s": B / (step_ms * 1e-3),
                      "GBps": B * (V * e + 4) / (step_ms * 1e-3) / 1e9, "round_trip": ok}), flush=True)
    coder.close()


if __name__ == "__main__":
    main()
