"""Self-describing container for lac bitstreams.

The reference writes bare bytes: ``measure_compress`` returns
``bytes(group_bits(bits))`` (arith_code.py:401-420) and stores neither the
symbol count n nor the bit length L, so its decoder cannot know where to stop
(arith_code.py:322-334; SURVEY.md finding 5).  This container adds a header in
front of exactly those bytes; the payload of each stream is unchanged.

Layout (little-endian):

    magic   4 B   b"LAC1"
    version u16   1
    prec    u8    coder precision (arith_code.py:157-160)
    flags   u8    bit0 mapping (0 ceil / CDFPredictor, 1 floor / Predictor, ACSampler)
                  bit1 termination (0 A_to_bin.flush, 1 ACSampler.flush_compress)
                  bit2 pmf_bits == 64
                  bit3 tables are q1-quantised logits (lac.h "logits path"): decode
                       needs the same logits, not a pmf
    vocab   u32
    streams u32
    then per stream: n_symbols u64, n_bits u64
    then per stream: ceil(n_bits / 8) payload bytes (MSB first, zero padded)
"""
from __future__ import annotations

import struct

MAGIC = b"LAC1"
VERSION = 1
_HDR = struct.Struct("<4sHBBII")
_ENT = struct.Struct("<QQ")


def pack(streams, n_symbols, n_bits, prec, vocab, mapping="ceil", termination="flush", pmf_bits=32,
         q1_logits=False) -> bytes:
    """streams: list of per-stream payload bytes (group_bits format)."""
    if not (len(streams) == len(n_symbols) == len(n_bits)):
        raise ValueError("streams, n_symbols and n_bits must have equal length")
    flags = ((mapping == "floor") | ((termination == "acsampler") << 1) | ((pmf_bits == 64) << 2)
             | (bool(q1_logits) << 3))
    out = [_HDR.pack(MAGIC, VERSION, prec, flags, vocab, len(streams))]
    for n, L, data in zip(n_symbols, n_bits, streams):
        if len(data) != (int(L) + 7) // 8:
            raise ValueError("payload length does not match n_bits")
        out.append(_ENT.pack(int(n), int(L)))
    out.extend(bytes(d) for d in streams)
    return b"".join(out)


def unpack(blob: bytes):
    """-> dict(prec, vocab, mapping, termination, pmf_bits, q1_logits, n_symbols, n_bits, streams)."""
    magic, ver, prec, flags, vocab, ns = _HDR.unpack_from(blob, 0)
    if magic != MAGIC:
        raise ValueError("not a LAC1 container")
    if ver != VERSION:
        raise ValueError(f"unsupported container version {ver}")
    off = _HDR.size
    n_symbols, n_bits = [], []
    for _ in range(ns):
        n, L = _ENT.unpack_from(blob, off)
        off += _ENT.size
        n_symbols.append(n)
        n_bits.append(L)
    streams = []
    for L in n_bits:
        k = (L + 7) // 8
        streams.append(blob[off:off + k])
        off += k
    if off != len(blob):
        raise ValueError("trailing bytes in container")
    return {"prec": prec, "vocab": vocab, "mapping": "floor" if flags & 1 else "ceil",
            "termination": "acsampler" if flags & 2 else "flush", "pmf_bits": 64 if flags & 4 else 32,
            "q1_logits": bool(flags & 8), "n_symbols": n_symbols, "n_bits": n_bits, "streams": streams}


def _is_logits(tables):
    import torch
    return tables.dtype in (torch.bfloat16, torch.float32)


def compress_batch(coder, pmf, sym) -> bytes:
    """Encode a batch with a BatchCoder and wrap it in a container.  ``pmf``:
    integer tables (one lac_encode_job) or bf16/f32 logits (the q1 logits path)."""
    logits = _is_logits(pmf)
    if logits:
        coder.encode_logits_job(pmf, sym)
    else:
        coder.encode_job(pmf, sym)
    data, nbits = coder.to_bytes()
    steps = sym.shape[0]
    return pack(data, [steps] * coder.streams, [int(x) for x in nbits], coder.prec, coder.vocab,
                pmf_bits=coder.pmf_bits, q1_logits=logits)


def decompress_batch(blob: bytes, pmf, device=None):
    """Decode a container produced by :func:`compress_batch` given the same tables
    (the same logits for a q1 container)."""
    import numpy as np
    import torch

    from .batch import BatchCoder
    h = unpack(blob)
    B = len(h["streams"])
    steps = max(h["n_symbols"]) if B else 0
    stride = max(8, ((max((len(s) for s in h["streams"]), default=0) + 7) // 8 + 1) * 8)
    buf = np.zeros((B, stride), dtype=np.uint8)
    for b, s in enumerate(h["streams"]):
        buf[b, :len(s)] = np.frombuffer(s, dtype=np.uint8)
    coder = BatchCoder(h["vocab"], B, prec=h["prec"], pmf_bits=h["pmf_bits"],
                       capacity_bits=max(h["n_bits"], default=64) + 64, device=device or pmf.device)
    coder.set_mapping(h["mapping"])
    bits = torch.from_numpy(buf).to(coder.device)
    nb = torch.tensor(h["n_bits"], dtype=torch.int64, device=coder.device)
    coder.decode_open(bits, nb)
    if h["q1_logits"] != _is_logits(pmf):
        raise ValueError("container and tables disagree: q1 logits vs integer pmf")
    out = coder.decode_logits(pmf[:steps]) if h["q1_logits"] else coder.decode(pmf[:steps])
    coder.raise_on_error()
    coder.close()
    return out, h["n_symbols"]
