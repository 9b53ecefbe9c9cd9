#!/usr/bin/env python3
"""Host-side split of the drop-in static decode (tools/dropin_bench.py's decode line):
``AC(CDFPredictor(list), 48).from_bin.run(bits, stop=0)`` at V=32000 on 10000 symbols.

    python tools/dropin_host_probe.py

Times, best of 5, in ms: the bit-list conversion (coder._bit_list), a fresh session with
its tables (_Session + load_bits + the row), a fresh BatchCoder (lac_open), one
decode_open + set_state, the whole run, and the device time of the decode kernels
(liblac hipEvents) for one whole run.  Prints one JSON line.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))


def best(fn, reps=5):
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return 1e3 * min(t)


def main():
    import numpy as np
    import torch
    import dropin_bench as db
    from oracle import oracle as coracle
    from lac_amd import coder as cm
    from lac_amd.batch import BatchCoder
    pmf = db.static_table()
    syms = db.draw(pmf, 10000, 5).tolist()
    cdf = np.cumsum(pmf).astype(np.int64).tolist()
    want, wL, _ = coracle.encode(pmf, syms, 48, static=True)
    bits = [int(b) for b in np.unpackbits(np.frombuffer(want, dtype=np.uint8))[:wL]]
    ac = cm.AC(cm.CDFPredictor(cdf), 48)
    list(ac.from_bin.run(bits, stop=0))                     # warm: library, device, kernels
    res = {"symbols": len(syms), "bits": wL}
    res["bit_list_ms"] = best(lambda: cm._bit_list(bits))
    bl, data = cm._bit_list(bits)

    def session():
        d = ac.from_bin
        s = cm._Session(d)
        s.load_bits(bl, data)
        s.tab.row()
        return s
    res["session_ms"] = best(session)
    res["batchcoder_open_close_ms"] = best(lambda: BatchCoder(32000, 1, prec=48, pmf_bits=64, capacity_bits=64).close())
    res["run_ms"] = best(lambda: list(ac.from_bin.run(bits, stop=0)))
    # device time of one run's decode kernels: profile the coder the session makes
    orig = cm._Session._coder_for
    holder = {}

    def hooked(self, V):
        c = orig(self, V)
        if "c" not in holder:
            holder["c"] = c
            c.lib.lac_profile_read(c.ctx, None, None, 1)
            c.lib.lac_profile_enable(c.ctx, 1)
        return c
    cm._Session._coder_for = hooked
    t0 = time.perf_counter()
    got = list(ac.from_bin.run(bits, stop=0))
    torch.cuda.synchronize()
    res["profiled_run_ms"] = 1e3 * (time.perf_counter() - t0)
    cm._Session._coder_for = orig
    c = holder["c"]
    ms = (C.c_double * 8)()
    cnt = (C.c_int64 * 8)()
    c.lib.lac_profile_read(c.ctx, C.cast(ms, C.c_void_p), C.cast(cnt, C.c_void_p), 1)
    res["decode_kernels_ms"] = ms[3]                        # KID_DECODE: stats path (stats + lean + seq)
    res["decode_launch_groups"] = int(cnt[3])
    res["ok"] = got[:len(syms)] == syms
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
