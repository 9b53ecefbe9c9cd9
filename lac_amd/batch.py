"""Batched device API: B independent streams coded on one MI355X.

This is the batched counterpart of the reference's single-stream coder
(``A_to_bin`` / ``A_from_bin``, /root/reference/arith_code.py:156-334) and of
``measure_compress`` (:401-420).  Tables stay in HBM as torch tensors; they
cross into liblac.so as raw device pointers (see include/lac.h).

    coder = BatchCoder(vocab=32000, streams=4096, prec=48)
    coder.encode(pmf, sym)           # pmf [steps, streams, V] uint32 in int32 storage
    coder.finish()
    data = coder.to_bytes()          # list of per-stream bytes (group_bits format)

    coder.decode_open()              # decode this coder's own output
    out = coder.decode(pmf)          # [steps, streams] int32 symbols
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import LacError, check



def _torch():
    import torch
    return torch


def _stream_handle(device):
    torch = _torch()
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


# include/lac.h lac_enc_state (EncState in lac_amd/csrc/lac_core.h)
ENC_STATE = np.dtype([("l", "<i8"), ("h", "<i8"), ("L", "<u8"), ("wa", "<u8"), ("wc", "<u8"), ("nsym", "<i8"),
                      ("err", "<i4"), ("nflush", "<i4"), ("err_step", "<i8"), ("flush", "i1", (8,))])


class StreamError(LacError):
    """A coder error on one or more streams (sticky, reported per stream)."""

    def __init__(self, code, err, err_step):
        first = int(np.flatnonzero(err)[0]) if np.any(err) else -1
        super().__init__(code, f"stream {first} failed at step {int(err_step[first]) if first >= 0 else -1}")
        self.err = err
        self.err_step = err_step
        self.first_stream = first


class BatchCoder:
    """Encoder/decoder for ``streams`` independent streams (one liblac context)."""

    def __init__(self, vocab: int, streams: int, prec: int = 48, pmf_bits: int = 32,
                 capacity_bits: int | None = None, device=None):
        torch = _torch()
        self.lib = _lib.load()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("BatchCoder needs a HIP device (torch 'cuda' device on ROCm)")
        self.vocab, self.streams, self.prec, self.pmf_bits = int(vocab), int(streams), int(prec), int(pmf_bits)
        self.capacity_bits = int(capacity_bits or 1 << 16)
        ctx = C.c_void_p()
        check(self.lib.lac_open(self.device.index or 0, self.prec, self.vocab, self.streams, self.pmf_bits,
                                self.capacity_bits, C.byref(ctx)))
        self.ctx = ctx

    # ------------------------------------------------------------ lifetime
    def close(self):
        if getattr(self, "ctx", None):
            self.lib.lac_close(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def _stream(self):
        return _stream_handle(self.device)

    # ------------------------------------------------------------ checks
    def _check_pmf(self, pmf):
        torch = _torch()
        want = (torch.int32, torch.uint32) if self.pmf_bits == 32 else (torch.int64, torch.uint64)
        if pmf.dtype not in want:
            raise TypeError(f"pmf must be {want[0]} (bit pattern of uint{self.pmf_bits}), got {pmf.dtype}")
        if pmf.device != self.device:
            raise ValueError(f"pmf is on {pmf.device}, coder on {self.device}")
        if pmf.shape[-1] != self.vocab:
            raise ValueError(f"pmf rows have {pmf.shape[-1]} entries, vocab is {self.vocab}")
        if pmf.stride(-1) != 1:
            raise ValueError("pmf rows must be contiguous")

    def _check_out(self, out, steps):
        torch = _torch()
        if out.dtype != torch.int32 or out.device != self.device:
            raise TypeError("out must be an int32 tensor on the coder's device")
        if tuple(out.shape) != (steps, self.streams) or not out.is_contiguous():
            raise ValueError(f"out must be a contiguous [{steps}, {self.streams}] tensor")

    # ------------------------------------------------------------ encode
    def reset(self):
        check(self.lib.lac_encode_reset(self.ctx, self._stream))

    def _encode_args(self, pmf, sym, trace):
        torch = _torch()
        self._check_pmf(pmf)
        if sym.dtype != torch.int32 or sym.device != self.device:
            raise TypeError("sym must be an int32 tensor on the coder's device")
        sym = sym.contiguous()
        steps = sym.shape[0] if sym.dim() == 2 else 1
        if sym.numel() != steps * self.streams:
            raise ValueError(f"sym must be [steps, {self.streams}]")
        if pmf.dim() == 1:
            step_stride, stream_stride = 0, 0
        elif pmf.dim() == 2:
            if steps != 1 or pmf.shape[0] != self.streams:
                raise ValueError("a 2-D pmf is [streams, V] for one step")
            step_stride, stream_stride = 0, pmf.stride(0)
        else:
            if pmf.shape[0] not in (1, steps) or pmf.shape[1] not in (1, self.streams):
                raise ValueError("pmf must be [steps, streams, V]")
            step_stride = pmf.stride(0) if pmf.shape[0] > 1 else 0
            stream_stride = pmf.stride(1) if pmf.shape[1] > 1 else 0
        tp = None
        if trace is not None:
            if trace.dtype != torch.int64 or trace.numel() != steps * self.streams * 2 or not trace.is_contiguous():
                raise ValueError("trace must be a contiguous int64 tensor [steps, streams, 2]")
            tp = C.c_void_p(trace.data_ptr())
        self._keep = (pmf, sym)
        return (self.ctx, C.c_void_p(pmf.data_ptr()), step_stride, stream_stride, C.c_void_p(sym.data_ptr()),
                steps, tp, self._stream)

    def encode(self, pmf, sym, trace=None):
        """Encode sym[t, b] with row pmf[t, b, :] (or pmf[b, :] / pmf[:] broadcast).

        ``pmf`` [steps, streams, V], [streams, V] (steps == 1), [V] (a static
        row for every step and stream) or [steps, 1, V] / [1, streams, V] with
        stride-0 broadcasting via ``expand``.  ``sym`` int32 [steps, streams].
        ``trace`` (optional int64 device tensor [steps, streams, 2]) receives
        per symbol {E, k} -- its raw digits.  Streams continue from where the
        previous call left them.
        """
        check(self.lib.lac_encode(*self._encode_args(pmf, sym, trace)))

    def encode_job(self, pmf, sym, trace=None):
        """reset + encode + finish in one call (one kernel at >= 2048 streams)."""
        check(self.lib.lac_encode_job(*self._encode_args(pmf, sym, trace)))

    def set_mapping(self, mapping):
        """'ceil' (CDFPredictor, default) or 'floor' (Predictor / ACSampler Region.map)."""
        v = {"ceil": _lib.LAC_MAP_CEIL, "floor": _lib.LAC_MAP_FLOOR}[mapping]
        check(self.lib.lac_set_option(self.ctx, _lib.LAC_OPT_MAPPING, v))

    def set_termination(self, term):
        """'flush' (A_to_bin.flush, default) or 'acsampler' (ACSampler.flush_compress)."""
        v = {"flush": _lib.LAC_TERM_FLUSH, "acsampler": _lib.LAC_TERM_ACSAMPLER}[term]
        check(self.lib.lac_set_option(self.ctx, _lib.LAC_OPT_TERMINATION, v))

    def set_decode_path(self, path):
        """'auto', 'split' (one workgroup per stream per step), 'fused' (one wave per
        stream, one launch; per-iteration row totals), 'fused_chunk' (the same with
        <= 64 chunk totals per row), 'stats' (all rows' chunk totals at once, then
        a sequential per-stream kernel) or 'block' (one workgroup per stream, the
        row scans pipelined a step ahead of the coder wave); identical results."""
        v = {"auto": _lib.LAC_PATH_AUTO, "split": _lib.LAC_PATH_SPLIT, "fused": _lib.LAC_PATH_FUSED,
             "fused_chunk": _lib.LAC_PATH_FUSED, "stats": _lib.LAC_PATH_STATS, "block": _lib.LAC_PATH_BLOCK}[path]
        check(self.lib.lac_set_option(self.ctx, _lib.LAC_OPT_DECODE_PATH, v))
        check(self.lib.lac_set_option(self.ctx, _lib.LAC_OPT_DECODE_FINE, 0 if path == "fused_chunk" else 1))

    def set_decode_stop(self, on: bool):
        """Stop each stream before the first symbol its bits do not determine (include/lac.h
        LAC_OPT_DECODE_STOP): its status becomes LAC_E_UNDETERMINED with the registers
        as they were before that symbol, where A_from_bin.run(bits, stop=0) stops
        (arith_code.py:268-299); decodes then take the stats path."""
        check(self.lib.lac_set_option(self.ctx, _lib.LAC_OPT_DECODE_STOP, 1 if on else 0))

    def set_block_waves(self, n: int):
        """Waves per stream of the 'block' decode path: 4, 8, 16 (0 = by stream count)."""
        check(self.lib.lac_set_option(self.ctx, _lib.LAC_OPT_BLOCK_WAVES, int(n)))

    def set_path(self, path):
        """'auto', 'split' or 'fused' encode kernels (bit-identical results)."""
        v = {"auto": _lib.LAC_PATH_AUTO, "split": _lib.LAC_PATH_SPLIT, "fused": _lib.LAC_PATH_FUSED}[path]
        check(self.lib.lac_set_option(self.ctx, _lib.LAC_OPT_ENCODE_PATH, v))

    def finish(self):
        check(self.lib.lac_encode_finish(self.ctx, self._stream))

    def rebase(self):
        """Drop every stream's completed output words, keeping its registers
        (include/lac.h lac_encode_rebase): for callers that take the digits from
        ``trace`` and only need the coder state to continue."""
        check(self.lib.lac_encode_rebase(self.ctx, self._stream))

    def status(self):
        err = np.zeros(self.streams, dtype=np.int32)
        step = np.zeros(self.streams, dtype=np.int64)
        rc = self.lib.lac_stream_status(self.ctx, err.ctypes.data_as(C.c_void_p), step.ctypes.data_as(C.c_void_p),
                                        self._stream)
        return rc, err, step

    def raise_on_error(self):
        rc, err, step = self.status()
        if rc:
            raise StreamError(rc, err, step)

    def registers(self):
        l = np.zeros(self.streams, dtype=np.int64)
        h = np.zeros(self.streams, dtype=np.int64)
        check(self.lib.lac_encoder_registers(self.ctx, l.ctypes.data_as(C.c_void_p), h.ctypes.data_as(C.c_void_p),
                                             self._stream))
        return l, h

    def checkpoint(self):
        """Everything the encoder holds (include/lac.h lac_encode_get_state): per-stream
        registers and counters (a numpy ENC_STATE array) and the output planes
        ([2, streams, cap_words] uint64).  restore() continues from it bit for bit."""
        st = np.zeros(self.streams, dtype=ENC_STATE)
        words = self.bits_stride() // 8
        planes = np.zeros((2, self.streams, words), dtype=np.uint64)
        check(self.lib.lac_encode_get_state(self.ctx, st.ctypes.data_as(C.c_void_p),
                                            planes.ctypes.data_as(C.c_void_p), self._stream))
        return {"state": st, "planes": planes, "prec": self.prec, "vocab": self.vocab}

    def restore(self, ckpt):
        """Load a checkpoint() of a coder with the same prec, vocab, streams and capacity."""
        st, planes = ckpt["state"], ckpt["planes"]
        if ckpt.get("prec", self.prec) != self.prec or ckpt.get("vocab", self.vocab) != self.vocab:
            raise ValueError("checkpoint of a coder with another prec / vocab")
        if st.dtype != ENC_STATE or st.shape != (self.streams,):
            raise ValueError(f"state must be ENC_STATE[{self.streams}]")
        if planes.dtype != np.uint64 or planes.shape != (2, self.streams, self.bits_stride() // 8):
            raise ValueError("planes of another capacity or stream count")
        st, planes = np.ascontiguousarray(st), np.ascontiguousarray(planes)
        check(self.lib.lac_encode_set_state(self.ctx, st.ctypes.data_as(C.c_void_p),
                                            planes.ctypes.data_as(C.c_void_p), self._stream))

    def lengths(self):
        n = np.zeros(self.streams, dtype=np.uint64)
        check(self.lib.lac_encoded_lengths(self.ctx, n.ctypes.data_as(C.c_void_p), self._stream))
        return n

    def device_bits(self):
        """(int pointer, stride_bytes, nbits pointer) of the packed output in HBM."""
        p, s, n = C.c_void_p(), C.c_uint64(), C.c_void_p()
        check(self.lib.lac_encoded_device(self.ctx, C.byref(p), C.byref(s), C.byref(n)))
        return p.value, s.value, n.value

    def bits_tensor(self, stride=None):
        """Packed output copied into a fresh uint8 device tensor [streams, stride]."""
        torch = _torch()
        _, s, _ = self.device_bits()
        stride = int(stride or s)
        out = torch.zeros((self.streams, stride), dtype=torch.uint8, device=self.device)
        check(self.lib.lac_copy_bits_dev(self.ctx, C.c_void_p(out.data_ptr()), stride, self._stream))
        return out

    def bits_stride(self):
        """Bytes per stream of the packed output buffer (capacity rounded to 8-byte words)."""
        return int(self.device_bits()[1])

    def copy_bits_into(self, out):
        """Copy the packed output into a uint8 device tensor [streams, W] with
        contiguous rows (W <= bits_stride() keeps the first W bytes), asynchronously."""
        if out.dim() != 2 or out.shape[0] != self.streams or out.stride(1) != 1 or out.dtype != _torch().uint8:
            raise ValueError("out must be a uint8 [streams, W] tensor with contiguous rows")
        check(self.lib.lac_copy_bits_dev(self.ctx, C.c_void_p(out.data_ptr()), out.stride(0), self._stream))
        return out

    def copy_nbits_into(self, out):
        """Copy the per-stream bit counts into a contiguous 8-byte integer device tensor [streams]."""
        if out.shape != (self.streams,) or not out.is_contiguous() or out.element_size() != 8:
            raise ValueError("out must be a contiguous 8-byte integer tensor [streams]")
        check(self.lib.lac_copy_nbits_dev(self.ctx, C.c_void_p(out.data_ptr()), self._stream))
        return out

    def pack_bits(self, out, hdr_bytes, length):
        """The finished streams packed for the wire into the uint8 device tensor ``out``
        (include/lac.h lac_pack_bits: a header of bit counts, ``hdr_bytes`` = 2 or 4 each,
        then each stream's bytes back to back); ``length`` (a one-element 8-byte integer
        device tensor) receives the packed length.  Asynchronous; no host sync."""
        if hdr_bytes not in (2, 4) or (hdr_bytes == 2 and self.bits_stride() * 8 >= 1 << 16):
            raise ValueError(f"hdr_bytes={hdr_bytes}: 2-byte headers need streams of < 65536 bits "
                             f"(this coder's hold {self.bits_stride() * 8}), else 4")
        need = self.streams * (hdr_bytes + self.bits_stride())
        if out.dtype != _torch().uint8 or not out.is_contiguous() or out.numel() < need or out.device != self.device:
            raise ValueError(f"out must be a contiguous uint8 device tensor of >= {need} bytes on {self.device}")
        if length.numel() != 1 or length.element_size() != 8 or length.device != self.device:
            raise ValueError("length must be a one-element 8-byte integer tensor on the coder's device")
        check(self.lib.lac_pack_bits(self.ctx, C.c_void_p(out.data_ptr()), int(hdr_bytes),
                                     C.c_void_p(length.data_ptr()), self._stream))
        return out, length

    def pack_bits_at(self, out, hdr_bytes, base, end, len_out=None):
        """pack_bits appended at byte offset ``base[0]`` of ``out`` (include/lac.h
        lac_pack_bits_at): ``base`` / ``end`` are one-element 8-byte integer device
        tensors (``base`` may be None: offset 0), ``end`` receives base + the packed
        length; ``len_out`` is None or a device address (int) of 8 bytes -- e.g. from
        lac_host_alloc -- for the packed length.  Asynchronous; no host sync."""
        if hdr_bytes not in (2, 4) or (hdr_bytes == 2 and self.bits_stride() * 8 >= 1 << 16):
            raise ValueError(f"hdr_bytes={hdr_bytes}: 2-byte headers need streams of < 65536 bits "
                             f"(this coder's hold {self.bits_stride() * 8}), else 4")
        if out.dtype != _torch().uint8 or not out.is_contiguous() or out.device != self.device:
            raise ValueError(f"out must be a contiguous uint8 device tensor on {self.device}")
        for t in (base, end):
            if t is not None and (t.numel() < 1 or t.element_size() != 8 or t.device != self.device):
                raise ValueError("base / end must be 8-byte integer tensors on the coder's device")
        check(self.lib.lac_pack_bits_at(self.ctx, C.c_void_p(out.data_ptr()), out.numel(), int(hdr_bytes),
                                        None if base is None else C.c_void_p(base.data_ptr()),
                                        C.c_void_p(end.data_ptr()),
                                        None if len_out is None else C.c_void_p(int(len_out)), self._stream))
        return out

    def set_output(self, planes=None, nbits=None):
        """Direct later encodes' output (plane A and the bit counts, include/lac.h
        lac_set_output) into caller-owned device tensors: ``planes`` of >= streams *
        cap_words + 1 int64 (``output_words()``), ``nbits`` of streams int64; None, None
        restores the coder's own.  The tensors are kept referenced while in use.
        Only between jobs: raises LacError(LAC_E_STATE) while a decode is open or an
        encode has coded symbols it has not finished (``encode`` since ``reset``, no
        ``finish`` yet).  Afterwards the coder counts as finished (``pack_bits``) only
        when the buffers are those its last finished job went to."""
        if (planes is None) != (nbits is None):
            raise ValueError("planes and nbits: both or neither")
        if planes is not None:
            for t, n in ((planes, self.output_words()), (nbits, self.streams)):
                if t.element_size() != 8 or not t.is_contiguous() or t.numel() < n or t.device != self.device:
                    raise ValueError(f"output buffers: contiguous 8-byte tensors of >= {n} elements on {self.device}")
        check(self.lib.lac_set_output(self.ctx, None if planes is None else C.c_void_p(planes.data_ptr()),
                                      None if nbits is None else C.c_void_p(nbits.data_ptr())))
        self._output = (planes, nbits)

    def output_words(self):
        """uint64 words of one job's plane A (set_output): streams * cap_words + 1."""
        return self.streams * (self.bits_stride() // 8) + 1

    def nbits_tensor(self):
        """Per-stream bit counts as a fresh int64 device tensor (asynchronous copy)."""
        torch = _torch()
        out = torch.empty((self.streams,), dtype=torch.int64, device=self.device)
        check(self.lib.lac_copy_nbits_dev(self.ctx, C.c_void_p(out.data_ptr()), self._stream))
        return out

    def to_bytes(self):
        """Per-stream bytes (MSB first, last byte zero padded: group_bits format)."""
        self.raise_on_error()
        n = self.lengths()
        _, s, _ = self.device_bits()
        host = np.zeros((self.streams, s), dtype=np.uint8)
        check(self.lib.lac_copy_bits(self.ctx, host.ctypes.data_as(C.c_void_p), s, self._stream))
        return [host[b, :(int(n[b]) + 7) // 8].tobytes() for b in range(self.streams)], n

    def flush_digits(self):
        d = np.zeros((self.streams, 8), dtype=np.int8)
        c = np.zeros(self.streams, dtype=np.int32)
        check(self.lib.lac_flush_digits(self.ctx, d.ctypes.data_as(C.c_void_p), c.ctypes.data_as(C.c_void_p),
                                        self._stream))
        return [d[b, :max(int(c[b]), 0)].tolist() for b in range(self.streams)]

    # ------------------------------------------------------------ decode
    def decode_open(self, bits=None, nbits=None):
        """Decode this coder's own output (no args), or ``bits`` (uint8 device
        tensor [streams, stride], stride % 8 == 0) with ``nbits`` (uint64/int64
        device tensor [streams])."""
        if bits is None:
            check(self.lib.lac_decode_open(self.ctx, None, 0, None, self._stream))
            self._dec_keep = None
            return
        torch = _torch()
        if bits.dtype != torch.uint8 or bits.device != self.device:
            raise TypeError("bits must be a uint8 tensor on the coder's device")
        if bits.dim() != 2 or bits.shape[0] != self.streams or bits.stride(1) != 1:
            raise ValueError("bits must be [streams, stride] with contiguous rows")
        if bits.stride(0) % 8 or bits.data_ptr() % 8:
            raise ValueError("bits rows must be 8-byte aligned (row stride a multiple of 8 bytes)")
        if nbits is None or nbits.dtype not in (torch.int64, torch.uint64) or nbits.device != self.device:
            raise TypeError("nbits must be an int64/uint64 tensor on the coder's device")
        if tuple(nbits.shape) != (self.streams,) or not nbits.is_contiguous():
            raise ValueError(f"nbits must be a contiguous [{self.streams}] tensor")
        # nbits[b] > 8 * stride fails that stream with a sticky LAC_E_ARG in the library
        self._dec_keep = (bits, nbits)                        # borrowed by the library
        check(self.lib.lac_decode_open(self.ctx, C.c_void_p(bits.data_ptr()), bits.stride(0),
                                       C.c_void_p(nbits.data_ptr()), self._stream))

    def determined(self):
        """Per stream: leading decoded symbols fixed by the available bits (the
        count the reference's A_from_bin.run(bits, stop=0) emits)."""
        n = np.zeros(self.streams, dtype=np.int64)
        check(self.lib.lac_decode_determined(self.ctx, n.ctypes.data_as(C.c_void_p), self._stream))
        return n

    def decode(self, pmf, out=None):
        """Decode one symbol per stream per step; pmf as in :meth:`encode`."""
        torch = _torch()
        self._check_pmf(pmf)
        if pmf.dim() == 2:
            pmf = pmf.unsqueeze(0)
        if pmf.dim() != 3:
            raise ValueError("give decode a [steps, streams, V] (or expanded) table")
        if pmf.shape[1] not in (1, self.streams):
            raise ValueError(f"pmf must be [steps, {self.streams} or 1, {self.vocab}], got {tuple(pmf.shape)}")
        steps = pmf.shape[0]
        step_stride = pmf.stride(0) if steps > 1 else 0
        stream_stride = pmf.stride(1) if pmf.shape[1] > 1 else 0
        if out is None:
            out = torch.empty((steps, self.streams), dtype=torch.int32, device=self.device)
        else:
            self._check_out(out, steps)
        check(self.lib.lac_decode_steps(self.ctx, C.c_void_p(pmf.data_ptr()), step_stride, stream_stride, steps,
                                        C.c_void_p(out.data_ptr()), self._stream))
        return out


    # ------------------------------------------------------------ logits path
    def _logits_args(self, logits, steps=None):
        """-> (type, step_stride, stream_stride, steps) for a [steps, streams, V]
        bf16/f32 logits tensor (stride-0 broadcasts allowed, rows contiguous)."""
        torch = _torch()
        typ = {torch.bfloat16: _lib.LAC_LOGITS_BF16, torch.float32: _lib.LAC_LOGITS_F32}.get(logits.dtype)
        if typ is None:
            raise TypeError(f"logits must be bfloat16 or float32, got {logits.dtype}")
        if logits.device != self.device:
            raise ValueError(f"logits are on {logits.device}, coder on {self.device}")
        if logits.dim() == 2:
            logits = logits.unsqueeze(0)
        if logits.dim() != 3 or logits.shape[1] not in (1, self.streams) or logits.shape[2] != self.vocab:
            raise ValueError(f"logits must be [steps, {self.streams}, {self.vocab}]")
        if logits.stride(2) != 1:
            raise ValueError("logit rows must be contiguous")
        n = logits.shape[0] if steps is None else steps
        if logits.shape[0] not in (1, n):
            raise ValueError("logits steps do not match the symbols")
        step_stride = logits.stride(0) if logits.shape[0] > 1 else 0
        stream_stride = logits.stride(1) if logits.shape[1] > 1 else 0
        return typ, step_stride, stream_stride, n, logits

    def _logits_encode_args(self, logits, sym, trace):
        torch = _torch()
        if sym.dtype != torch.int32 or sym.device != self.device:
            raise TypeError("sym must be an int32 tensor on the coder's device")
        sym = sym.contiguous()
        steps = sym.shape[0] if sym.dim() == 2 else 1
        if sym.numel() != steps * self.streams:
            raise ValueError(f"sym must be [steps, {self.streams}]")
        typ, ss, bs, steps, logits = self._logits_args(logits, steps)
        tp = None
        if trace is not None:
            if trace.dtype != torch.int64 or trace.numel() != steps * self.streams * 2 or not trace.is_contiguous():
                raise ValueError("trace must be a contiguous int64 tensor [steps, streams, 2]")
            tp = C.c_void_p(trace.data_ptr())
        self._keep = (logits, sym)
        return (self.ctx, C.c_void_p(logits.data_ptr()), typ, ss, bs, C.c_void_p(sym.data_ptr()), steps, tp,
                self._stream)

    def encode_logits(self, logits, sym, trace=None):
        """Incremental logits encode: continue every stream by ``steps`` symbols
        (no reset, no finish -- call :meth:`finish` at the end).  Steps may be
        interleaved with :meth:`encode` on integer pmfs."""
        check(self.lib.lac_encode_logits(*self._logits_encode_args(logits, sym, trace)))

    def encode_logits_job(self, logits, sym, trace=None):
        """reset + encode + finish with tables computed in-kernel from logits by
        the q1 quantiser (include/lac.h "logits path"): the pmf never touches
        HBM.  ``logits`` [steps, streams, V] bf16/f32, ``sym`` [steps, streams]."""
        check(self.lib.lac_encode_logits_job(*self._logits_encode_args(logits, sym, trace)))

    def decode_logits(self, logits, out=None):
        """Decode one symbol per stream per step with q1 tables from ``logits``."""
        torch = _torch()
        typ, ss, bs, steps, logits = self._logits_args(logits)
        if out is None:
            out = torch.empty((steps, self.streams), dtype=torch.int32, device=self.device)
        else:
            self._check_out(out, steps)
        check(self.lib.lac_decode_logits_steps(self.ctx, C.c_void_p(logits.data_ptr()), typ, ss, bs, steps,
                                               C.c_void_p(out.data_ptr()), self._stream))
        return out

    def quantize_logits(self, logits):
        """The q1 tables themselves: int32 tensor (uint32 bit patterns) [steps, streams, V]."""
        torch = _torch()
        typ, ss, bs, steps, logits = self._logits_args(logits)
        out = torch.empty((steps, self.streams, self.vocab), dtype=torch.int32, device=self.device)
        check(self.lib.lac_quantize_logits(self.ctx, C.c_void_p(logits.data_ptr()), typ, ss, bs, steps,
                                           C.c_void_p(out.data_ptr()), self._stream))
        return out

    def set_q1_shape(self, shape: int):
        """Logits row-stats block shape (include/lac.h LAC_OPT_Q1_SHAPE; identical
        results, only speed differs): 0 auto, 1..4 / 6 / 8 / 10 / 14 / 15 / 17 / 18
        forced single-block forms, 19 / 20 / 21 row groups -- a row of > 16384
        vectors in 2..16 segments, one per row slot of 1 / 2 / 4 rows per 16-wave
        block --, 22 one row of <= 26112 vectors in the registers (+ LDS slots) of
        one 8-wave block, 23 groups of such blocks.  The retired shapes 5, 7, 9, 11,
        12, 13 and 16 (never chosen by AUTO) raise LacError (LAC_E_ARG)."""
        check(self.lib.lac_set_option(self.ctx, _lib.LAC_OPT_Q1_SHAPE, int(shape)))

    def q1_k(self):
        """The q1 table scale: max entry 2^k, k = min(24, prec - 1 - ceil(log2 V)) (lac.h lac_q1_k)."""
        return int(self.lib.lac_q1_k(self.prec, self.vocab))


def logits_row_multiple(dtype) -> int:
    """Entries per 16-B vector of a logits row (8 bf16, 4 f32): the logits path
    (lac_encode_logits, include/lac.h) needs vocab and row strides to be multiples of it."""
    torch = _torch()
    if dtype not in (torch.bfloat16, torch.float32):
        raise TypeError(f"logits must be bfloat16 or float32, got {dtype}")
    return 8 if dtype == torch.bfloat16 else 4


def pad_logits(logits):
    """[..., V] logits -> contiguous [..., Vp] with Vp the next multiple of
    logits_row_multiple, the new entries -inf (q1 gives each the minimum weight, 1).
    Encode and decode must both code the padded rows."""
    torch = _torch()
    m = logits_row_multiple(logits.dtype)
    V = logits.shape[-1]
    Vp = (V + m - 1) // m * m
    if Vp != V:
        logits = torch.nn.functional.pad(logits, (0, Vp - V), value=float("-inf"))
    return logits.contiguous()


def digits_of(E: int, k: int):
    """Raw digits of one symbol from its trace entry (first digit 0..3)."""
    if k <= 0:
        return []
    return [E >> (k - 1)] + [(E >> (k - 1 - i)) & 1 for i in range(1, k)]
