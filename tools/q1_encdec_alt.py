#!/usr/bin/env python3
"""Logits-path encode and decode alternated on one job (tuning aid): the q1 row-stats
kernel's device time in each direction, per repetition, to separate the decode form's
own cost from ordering / clock effects.

    python tools/q1_encdec_alt.py [--vocab 128256] [--input logits-bf16] [--reps 4]
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--vocab", type=int, default=128256)
    ap.add_argument("--streams", type=int, default=4096)
    ap.add_argument("--tokens", type=int, default=16)
    ap.add_argument("--input", default="logits-bf16")
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--q1-shape", type=int, default=0)
    a = ap.parse_args()
    import torch
    from lac_amd import synth
    from lac_amd.batch import BatchCoder
    dev = torch.device("cuda", 0)
    V, B, T = a.vocab, a.streams, a.tokens
    coder = BatchCoder(V, B, prec=48, capacity_bits=T * 50 + 256, device=dev)
    if a.q1_shape:
        coder.set_q1_shape(a.q1_shape)
    dt = torch.bfloat16 if a.input == "logits-bf16" else torch.float32
    lg, sym = synth.logits_batch(T, B, V, device=dev, dtype=dt, quantise=coder.quantize_logits)
    ms = (C.c_double * 8)()
    cnt = (C.c_int64 * 8)()

    def timed(fn):
        torch.cuda.synchronize()
        coder.lib.lac_profile_read(coder.ctx, None, None, 1)
        coder.lib.lac_profile_enable(coder.ctx, 1)
        r = fn()
        torch.cuda.synchronize()
        coder.lib.lac_profile_enable(coder.ctx, 0)
        coder.lib.lac_profile_read(coder.ctx, C.cast(ms, C.c_void_p), C.cast(cnt, C.c_void_p), 1)
        return r, ms[6], ms[7]

    res = []
    for i in range(a.reps):
        _, e6, _ = timed(lambda: coder.encode_logits_job(lg, sym))
        coder.decode_open()
        out, d6, d7 = timed(lambda: coder.decode_logits(lg))
        res.append({"enc_stats_ms": e6, "dec_stats_ms": d6, "dec_seq_ms": d7, "ok": bool(torch.equal(out, sym))})
        print(json.dumps(res[-1]), flush=True)


if __name__ == "__main__":
    main()
