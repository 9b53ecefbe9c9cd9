#!/usr/bin/env python3
"""Logits-path row statistics, encode vs decode form, each timed over back-to-back
launches with no host synchronisation in between (so neither pays a clock ramp after
an idle gap): per-launch device time of k_q1_stats (liblac hipEvents) in both forms.

    python tools/q1_b2b.py --vocab 151936 [--reps 10] [--q1-shape 0]
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--vocab", type=int, default=151936)
    ap.add_argument("--streams", type=int, default=4096)
    ap.add_argument("--tokens", type=int, default=16)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--q1-shape", type=int, default=0)
    ap.add_argument("--dtype", default="bf16")
    a = ap.parse_args()
    import torch
    from lac_amd import synth
    from lac_amd.batch import BatchCoder
    dev = torch.device("cuda", 0)
    V, B, T, P = a.vocab, a.streams, a.tokens, 48
    coder = BatchCoder(V, B, prec=P, pmf_bits=32, capacity_bits=T * (P + 2) + 256, device=dev)
    if a.q1_shape:
        coder.set_q1_shape(a.q1_shape)
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    logits, sym = synth.logits_batch(T, B, V, seed=1234, device=dev, dtype=dt, quantise=coder.quantize_logits)
    lib = coder.lib
    ms = (C.c_double * 8)()
    cnt = (C.c_int64 * 8)()
    eb = T * B * (V * logits.element_size() + 4)
    res = {"vocab": V, "dtype": a.dtype, "q1_shape": a.q1_shape}
    for phase in ("encode", "decode", "encode2", "decode2"):
        for _ in range(3):                                   # warm, back to back
            if phase.startswith("encode"):
                coder.encode_logits_job(logits, sym)
            else:
                coder.decode_open()
                coder.decode_logits(logits)
        lib.lac_profile_read(coder.ctx, None, None, 1)
        lib.lac_profile_enable(coder.ctx, 1)
        out = None
        for _ in range(a.reps):
            if phase.startswith("encode"):
                coder.encode_logits_job(logits, sym)
            else:
                coder.decode_open()
                out = coder.decode_logits(logits)
        torch.cuda.synchronize()
        lib.lac_profile_enable(coder.ctx, 0)
        lib.lac_profile_read(coder.ctx, C.cast(ms, C.c_void_p), C.cast(cnt, C.c_void_p), 1)
        per = ms[6] / max(cnt[6], 1)
        res[phase] = {"q1_stats_ms_per_launch": per, "launches": int(cnt[6]),
                      "frac_of_8TBps": eb / (per * 1e-3) / 8e12 if per else None,
                      "q1_decode_us_per_step": 1e3 * ms[7] / max(a.reps * T, 1) if cnt[7] else None}
        if out is not None:
            res[phase]["round_trip"] = bool(torch.equal(out, sym))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
