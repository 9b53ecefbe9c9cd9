"""Row-group launches (f32 V=128256, shape 19) while tests/native/hog.hip holds
half the CUs: wall time of the encode job, whether it aborted, bytes equal."""
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lac_amd import _lib  # noqa: E402
from lac_amd.batch import BatchCoder  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
hog = C.CDLL(os.path.join(REPO, "tests", "native", "libhog.so"))
hog.hog_launch.argtypes = [C.c_int, C.c_double, C.c_void_p, C.c_void_p]
DEV = "cuda:0"
V, B, steps, prec = 128256, 256, 2, 48
x = torch.randn((steps, B, V), device=DEV) * 3
sym = torch.randint(0, V, (steps, B), device=DEV, dtype=torch.int32)
c = BatchCoder(V, B, prec=prec, pmf_bits=32, capacity_bits=steps * 50 + 256, device=DEV)
c.encode_logits_job(x, sym)
want, _ = c.to_bytes()
ok = torch.zeros(1, dtype=torch.int32, device=DEV)
busy, mine = torch.cuda.Stream(device=DEV), torch.cuda.Stream(device=DEV)
cus = torch.cuda.get_device_properties(0).multi_processor_count
for nh in (cus - 8,):
    for hs in (0.0, 0.2, 0.6, 1.5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if hs:
            hog.hog_launch(nh, hs, C.c_void_p(ok.data_ptr()), C.c_void_p(busy.cuda_stream))
            time.sleep(0.05)
        t1 = time.perf_counter()
        with torch.cuda.stream(mine):
            c.encode_logits_job(x, sym)
            mine.synchronize()
            t2 = time.perf_counter()
            ab = C.c_int64()
            _lib.check(c.lib.lac_q1_group_aborted(c.ctx, C.byref(ab), c._stream))
            got, _ = c.to_bytes()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        print(f"hog {hs:.2f}s on {nh} CUs: encode wall {1e3 * (t2 - t1):8.1f} ms, all done "
              f"{1e3 * (t3 - t0):8.1f} ms, aborted={ab.value}, equal={got == want}", flush=True)
        if hs:
            hog.hog_launch(nh, hs, C.c_void_p(ok.data_ptr()), C.c_void_p(busy.cuda_stream))
            time.sleep(0.05)
        t1 = time.perf_counter()
        with torch.cuda.stream(mine):
            c.decode_open()
            dec = c.decode_logits(x)
            mine.synchronize()
            t2 = time.perf_counter()
            ab = C.c_int64()
            _lib.check(c.lib.lac_q1_group_aborted(c.ctx, C.byref(ab), c._stream))
        torch.cuda.synchronize()
        print(f"          decode wall {1e3 * (t2 - t1):8.1f} ms, aborted={ab.value}, equal={torch.equal(dec, sym)}",
              flush=True)
