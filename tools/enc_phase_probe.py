#!/usr/bin/env python3
"""Where one few-stream encode step spends its time: the c2
workload (V=32000, 1 stream, T steps) encoded by the split path (k_row_stats, then
k_encode's serial chain) with a probe build of liblac (-DLAC_ENC_PHASES=1:
    python3 -m lac_amd.build --out tools/_probe/liblac_encphases.so -DLAC_ENC_PHASES=1)
whose k_encode adds s_memtime marks between the phases of the sequential step:

  0 the step's stats out of the prefetch lanes (8 readlanes), the symbol, the row pointer
  1 the range: fudge test and two ceil mul-divs through the row fractions
  2 narrowing and renormalisation (k, E)
  3 appending E's bits and carry to the planes
  4 the per-64-step prefetch block (stats loads, row fractions, fudge thresholds)

    LAC_LIB=tools/_probe/liblac_encphases.so python tools/enc_phase_probe.py [--tokens 4096]

Prints one JSON line: shader cycles per step per phase (the marks cost a few cycles
each) and the encode kernels' hipEvent time per step for scale.
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
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--one-generator", action="store_true",
                    help="tables from one torch generator (for runs under rocprofv3 --pmc)")
    a = ap.parse_args()
    import torch
    from lac_amd import synth
    from lac_amd.batch import BatchCoder
    dev = torch.device("cuda", 0)
    V, B, T, P = a.vocab, a.streams, a.tokens, 48
    coder = BatchCoder(V, B, prec=P, pmf_bits=32, capacity_bits=T * (P + 2) + 256, device=dev)
    if a.one_generator:                     # (for runs under rocprofv3 --pmc: tools/probe_tables.py)
        from tools.probe_tables import one_generator_tables
        pmf, sym = one_generator_tables(T, B, V, dev)
    else:
        pmf, sym = synth.softmax_tables(T, B, V, seed=1234, device=dev, scale_bits=31, storage_bits=32)
    lib = coder.lib
    probe = hasattr(lib, "lac_debug_enc_phases")
    out = (C.c_uint64 * 8)()
    if probe:
        lib.lac_debug_enc_phases.argtypes = [C.c_void_p, C.c_int]
    names = ["stats_readlanes", "range_muldiv", "narrow_renorm", "plane_append", "prefetch_block"]
    res = {}
    for rep in range(a.reps):
        if probe:
            lib.lac_debug_enc_phases(C.cast(out, C.c_void_p), 1)
        ms = (C.c_double * 8)()
        cnt = (C.c_int64 * 8)()
        lib.lac_profile_read(coder.ctx, None, None, 1)
        lib.lac_profile_enable(coder.ctx, 1)
        coder.encode_job(pmf, sym)
        torch.cuda.synchronize()
        lib.lac_profile_enable(coder.ctx, 0)
        lib.lac_profile_read(coder.ctx, C.cast(ms, C.c_void_p), C.cast(cnt, C.c_void_p), 1)
        res = {"rep": rep, "kernel_us_per_step": {"row_stats": 1e3 * ms[0] / T, "encode": 1e3 * ms[1] / T,
                                                  "finish": 1e3 * ms[2] / T}}
        if probe:
            lib.lac_debug_enc_phases(C.cast(out, C.c_void_p), 1)
            steps = max(int(out[6]), 1)
            cyc = {n: out[k] / steps for k, n in enumerate(names)}
            res.update({"steps": steps, "cycles_per_step": cyc, "cycles_total_per_step": sum(cyc.values())})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
