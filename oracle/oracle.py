"""ctypes front for the C oracle (liblacref.so) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module; it is the checker, never the thing measured or shipped.
Build: ``make -C oracle`` (done by ``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liblacref.so")

_u8p = C.POINTER(C.c_uint8)
_lib = None


def build():
    import subprocess
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.lacref_encode.restype = C.c_int
        L.lacref_encode.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_int64, C.c_int64, C.c_void_p,
                                    C.c_int, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint64,
                                    C.c_void_p, C.c_void_p]
        L.lacref_encode_batch.restype = C.c_int
        L.lacref_encode_batch.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_int64, C.c_int64, C.c_int64,
                                          C.c_int64, C.c_void_p, C.c_int, C.c_void_p, C.c_uint64,
                                          C.c_void_p, C.c_void_p, C.c_int]
        L.lacref_decode.restype = C.c_int
        L.lacref_decode.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_int64, C.c_int64, C.c_void_p,
                                    C.c_uint64, C.c_int, C.c_void_p]
        L.lacref_decode_bitserial.restype = C.c_int64
        L.lacref_decode_bitserial.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_int64, C.c_int64, C.c_void_p,
                                              C.c_uint64, C.c_int, C.c_void_p, C.c_int64]
        L.lacref_q1_quantize.restype = C.c_int
        L.lacref_q1_quantize.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_int, C.c_void_p]
        L.lacref_q1_k.restype = C.c_int
        L.lacref_q1_k.argtypes = [C.c_int, C.c_int64]
        L.lacref_acsampler_encode.restype = C.c_int
        L.lacref_acsampler_encode.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int,
                                              C.c_void_p, C.c_uint64, C.c_void_p]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def _rows_array(rows):
    """rows: 2-D array-like [steps][V] of ints -> contiguous uint32/uint64 array."""
    a = np.asarray(rows)
    if a.dtype == object or a.dtype.kind == "i" or a.dtype.kind == "u":
        mx = max((int(x) for x in np.ravel(a)), default=0)
        dt = np.uint32 if mx < 2 ** 32 and a.dtype != np.uint64 else np.uint64
        a = np.array([[int(x) for x in r] for r in a], dtype=dt) if a.dtype == object else a.astype(dt)
    return np.ascontiguousarray(a)


class OracleError(RuntimeError):
    def __init__(self, code, step=None):
        super().__init__(f"oracle status {code}" + (f" at step {step}" if step is not None else ""))
        self.code = code
        self.step = step


def encode(rows, syms, prec, static=False):
    """-> (bytes, nbits, digits).  ``rows`` [steps][V] (or one row with static=True)."""
    a = _rows_array(rows if not static else [rows])
    s = np.ascontiguousarray(np.asarray(syms, dtype=np.int32))
    steps = len(s)
    V = a.shape[1]
    cap_d = steps * (prec + 2) + 64
    out = np.zeros(cap_d // 8 + 16, dtype=np.uint8)
    dig = np.zeros(cap_d, dtype=np.int8)
    nbits = np.zeros(1, dtype=np.uint64)
    nd = np.zeros(1, dtype=np.uint64)
    fail = np.full(1, -1, dtype=np.int64)
    stride = 0 if static or a.shape[0] == 1 else V
    if a.shape[0] != 1 and not static and a.shape[0] < steps:
        raise ValueError("fewer rows than symbols")
    rc = lib().lacref_encode(_ptr(a), a.itemsize, V, steps, stride, _ptr(s), prec, _ptr(out), out.size,
                             _ptr(nbits), _ptr(dig), dig.size, _ptr(nd), _ptr(fail))
    if rc:
        raise OracleError(rc, int(fail[0]))
    L = int(nbits[0])
    return out[:(L + 7) // 8].tobytes(), L, dig[:int(nd[0])].tolist()


def encode_batch(pmf, syms, prec, nthreads=1, cap_bytes=None):
    """pmf [steps][streams][V] (uint32/uint64), syms [steps][streams] -> (out[streams,cap], nbits[streams])."""
    pmf = np.ascontiguousarray(pmf)
    syms = np.ascontiguousarray(syms, dtype=np.int32)
    steps, streams, V = pmf.shape
    if cap_bytes is None:
        cap_bytes = (steps * (prec + 2) + 64) // 8 + 16
    out = np.zeros((streams, cap_bytes), dtype=np.uint8)
    nbits = np.zeros(streams, dtype=np.uint64)
    status = np.zeros(streams, dtype=np.int32)
    rc = lib().lacref_encode_batch(_ptr(pmf), pmf.itemsize, V, steps, streams, streams * V, V, _ptr(syms),
                                   prec, _ptr(out), cap_bytes, _ptr(nbits), _ptr(status), nthreads)
    return out, nbits, status, rc


def decode(rows, data: bytes, nbits: int, nsym: int, prec: int, static=False):
    a = _rows_array(rows if not static else [rows])
    V = a.shape[1]
    stride = 0 if static or a.shape[0] == 1 else V
    buf = np.frombuffer(bytes(data) + b"\0" * 8, dtype=np.uint8).copy()
    out = np.zeros(max(nsym, 1), dtype=np.int32)
    rc = lib().lacref_decode(_ptr(a), a.itemsize, V, nsym, stride, _ptr(buf), nbits, prec, _ptr(out))
    if rc:
        raise OracleError(rc)
    return out[:nsym].tolist()


def decode_bitserial(rows, data: bytes, nbits: int, prec: int, max_out: int = 1 << 20):
    """A_from_bin.run(bits, stop=0) (the reference's bit-serial decoder, literal in
    C): every symbol the bits determine; rows[min(t, len-1)] for step t."""
    a = _rows_array(rows)
    V = a.shape[1]
    buf = np.frombuffer(bytes(data) + b"\0" * 8, dtype=np.uint8).copy()
    out = np.zeros(max(max_out, 1), dtype=np.int32)
    n = lib().lacref_decode_bitserial(_ptr(a), a.itemsize, V, a.shape[0], V, _ptr(buf), nbits, prec, _ptr(out),
                                      max_out)
    if n < 0:
        raise OracleError(int(n))
    return out[:min(n, max_out)].tolist()


def acsampler_encode(cdf, tokens, prec=48):
    c = np.ascontiguousarray(np.asarray([int(x) for x in cdf], dtype=np.uint64))
    t = np.ascontiguousarray(np.asarray(tokens, dtype=np.int32))
    cap = len(t) * (prec + 2) + 256
    out = np.zeros(cap, dtype=np.uint8)
    n = np.zeros(1, dtype=np.uint64)
    rc = lib().lacref_acsampler_encode(_ptr(c), len(c), _ptr(t), len(t), prec, _ptr(out), cap, _ptr(n))
    if rc:
        raise OracleError(rc)
    return out[:int(n[0])].tolist()


def q1_quantize(logits, prec):
    """q1 quantiser (C oracle) over rows of bf16 (numpy uint16 bit patterns) or
    float32 logits, any leading shape -> uint32 pmf of the same shape."""
    x = np.ascontiguousarray(logits)
    typ = 1 if x.dtype == np.uint16 else 2
    if typ == 2:
        x = x.astype(np.float32)
    V = x.shape[-1]
    flat = x.reshape(-1, V)
    out = np.zeros(flat.shape, dtype=np.uint32)
    for r in range(flat.shape[0]):
        rc = lib().lacref_q1_quantize(_ptr(flat[r]), typ, V, prec, _ptr(out[r]))
        if rc:
            raise OracleError(rc)
    return out.reshape(x.shape)
