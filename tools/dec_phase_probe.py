#!/usr/bin/env python3
"""Where one few-stream decode step spends its time: the c2
workload (V=32000, 1 stream, T steps) decoded by the stats path with a probe build
of liblac (-DLAC_DEC_PHASES=1, tools/dec_phase_probe.sh) whose k_decode_seq adds
s_memtime marks between the phases of the sequential step:

  0 row totals + their wave scan (loop top, prefetch of the next row's totals)
  1 targets floor(v*T/w) (and the 1-padded twin)
  2 chunk search (ballot over the 64 chunk totals)
  3 re-read of the target chunk (one round of loads) + its scan to the symbol
  4 ranges ceil(c*w/T)
  5 narrowing, renormalisation, bit window

    LAC_LIB=tools/_probe/liblac_phases.so python tools/dec_phase_probe.py [--tokens 4096]

Prints one JSON line: shader cycles per step per phase (the marks cost a few
cycles each) and the decode kernels' hipEvent time per step for scale.
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--vocab", type=int, default=32000)
    ap.add_argument("--tokens", type=int, default=4096)
    ap.add_argument("--streams", type=int, default=1)
    ap.add_argument("--kernel", default="lean", choices=("lean", "seq"),
                    help="which sequential kernel the probe library runs (seq: a -DLAC_LEAN=0 build)")
    ap.add_argument("--pmf-bits", type=int, default=32, choices=(32, 64),
                    help="table storage; 64: llama-scale u64 tables (max(2, floor(softmax * 2^60)))")
    ap.add_argument("--scale-bits", type=int, default=0,
                    help="softmax scale of the tables (default 31 for u32, 60 for u64; e.g. 40: u64 totals ~2^40)")
    ap.add_argument("--static", action="store_true",
                    help="one row for every step (stride 0): the drop-in surface's static model")
    ap.add_argument("--one-generator", action="store_true",
                    help="tables from one torch generator (for runs under rocprofv3 --pmc)")
    a = ap.parse_args()
    import torch
    from lac_amd import synth
    from lac_amd.batch import BatchCoder
    dev = torch.device("cuda", 0)
    V, B, T, P = a.vocab, a.streams, a.tokens, 48
    coder = BatchCoder(V, B, prec=P, pmf_bits=a.pmf_bits, capacity_bits=T * (P + 2) + 256, device=dev)
    if a.one_generator:                     # (for runs under rocprofv3 --pmc: tools/probe_tables.py)
        from tools.probe_tables import one_generator_tables
        pmf, sym = one_generator_tables(T, B, V, dev)
    else:
        pmf, sym = synth.softmax_tables(T, B, V, seed=1234, device=dev, scale_bits=a.scale_bits or (31 if a.pmf_bits == 32 else 60),
                                        storage_bits=a.pmf_bits)
    if a.static:                            # the first step's rows for every step, symbols drawn from them
        row = pmf[:1]
        cdf = torch.cumsum(row[0].to(torch.int64) & (0xFFFFFFFF if a.pmf_bits == 32 else -1), dim=-1)
        g = torch.Generator(device=dev).manual_seed(5)
        u = torch.rand((T, B), generator=g, device=dev, dtype=torch.float64)
        tgt = (u * cdf[:, -1].double()[None]).floor().long().clamp(max=int(cdf[:, -1].min()) - 1)
        sym = torch.stack([torch.searchsorted(cdf[b], tgt[:, b].contiguous(), right=True) for b in range(B)], 1)
        sym = sym.to(torch.int32).contiguous()
        pmf = row.expand(T, B, V)
    coder.encode_job(pmf, sym)
    lib = coder.lib
    probe = hasattr(lib, "lac_debug_dec_phases")     # (a plain library: kernel times only)
    if probe:
        lib.lac_debug_dec_phases.argtypes = [C.c_void_p, C.c_int]
    out = (C.c_uint64 * 8)()
    res = {}
    for rep in range(3):
        coder.decode_open()
        if probe:
            lib.lac_debug_dec_phases(C.cast(out, C.c_void_p), 1)
        ms = (C.c_double * 8)()
        cnt = (C.c_int64 * 8)()
        lib.lac_profile_read(coder.ctx, None, None, 1)
        lib.lac_profile_enable(coder.ctx, 1)
        dec = coder.decode(pmf)
        torch.cuda.synchronize()
        lib.lac_profile_enable(coder.ctx, 0)
        lib.lac_profile_read(coder.ctx, C.cast(ms, C.c_void_p), C.cast(cnt, C.c_void_p), 1)
        if probe:
            lib.lac_debug_dec_phases(C.cast(out, C.c_void_p), 1)
        steps = max(int(out[6]), 1)
        names = (["top", "chunk+load_issue+target", "past", "wait+iteration+search", "ranges+exit",
                  "advance+output"] if a.kernel == "lean" else
                 ["totals+scan", "targets", "chunk_search", "reread+scan", "ranges", "renorm"])
        cyc = {n: out[k] / steps for k, n in enumerate(names)}
        res = {"rep": rep, "steps": steps, "cycles_per_step": cyc, "cycles_total_per_step": sum(cyc.values()),
               "kernel_us_per_step": {"decode (stats + seq)": 1e3 * ms[3] / max(T, 1)},
               "round_trip": bool(torch.equal(dec, sym))}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
