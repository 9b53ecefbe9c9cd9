#!/usr/bin/env python3
"""Which forced q1 row-stats shapes reproduce the AUTO bytes at a given (V, dtype)?
    python3 tools/q1_shape_check.py V bf16|f32"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_gpu_logits import _coder, _device_logits, _logits, _sample  # noqa: E402

from lac_amd._lib import LacError  # noqa: E402

V, dtype = int(sys.argv[1]), sys.argv[2]
B, steps, prec = 12, 3, 48
x = _logits(777, steps, B, V, specials=True)
dl = _device_logits(x, dtype)
c = _coder(V, B, prec, cap=steps * (prec + 2) + 256)
pmf = c.quantize_logits(dl).cpu().numpy().view(np.uint32)
sym = torch.from_numpy(_sample(pmf, 5)).to("cuda:0")
from oracle import oracle as coracle  # noqa: E402
out, nb, _, rc = coracle.encode_batch(pmf, sym.cpu().numpy(), prec, nthreads=8)
want = [out[b, :(int(nb[b]) + 7) // 8].tobytes() for b in range(B)]
for sh in range(0, 24):
    try:
        c.set_q1_shape(sh)
        c.encode_logits_job(dl, sym)
    except LacError as e:
        print(sh, "refused", e)
        continue
    rc, err, step = c.status()
    if rc:
        print(sh, "stream errors", err.tolist()[:4])
        continue
    got, gn = c.to_bytes()
    ok = got == want
    c.decode_open()
    dok = torch.equal(c.decode_logits(dl), sym)
    print(sh, "encode", "OK" if ok else "MISMATCH", "decode", "OK" if dok else "MISMATCH", flush=True)
