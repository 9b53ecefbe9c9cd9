"""ctypes binding of liblac.so (include/lac.h).

The library is built in-tree (``python -m lac_amd.build`` or
``__graft_entry__.build()``) and loaded from ``lac_amd/liblac.so``.  There is no
fallback: if the library is missing or fails to load, every coder entry point
raises :class:`LacLibraryError`.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LAC_LIB") or os.path.join(HERE, "liblac.so")   # LAC_LIB: tuning variants only

LAC_OK = 0
LAC_E_ARG = -1
LAC_E_PREC = -2
LAC_E_SYMBOL_RANGE = -3
LAC_E_ZERO_WIDTH = -4
LAC_E_TABLE = -5
LAC_E_DECODE_RANGE = -6
LAC_E_CAPACITY = -7
LAC_E_HIP = -8
LAC_E_STATE = -9
LAC_E_FLUSH_ZERO_WIDTH = -10
LAC_E_FLUSH_LOOP = -11
LAC_E_UNDETERMINED = -12

STATUS_NAMES = {
    LAC_OK: "LAC_OK", LAC_E_ARG: "LAC_E_ARG", LAC_E_PREC: "LAC_E_PREC",
    LAC_E_SYMBOL_RANGE: "LAC_E_SYMBOL_RANGE", LAC_E_ZERO_WIDTH: "LAC_E_ZERO_WIDTH",
    LAC_E_TABLE: "LAC_E_TABLE", LAC_E_DECODE_RANGE: "LAC_E_DECODE_RANGE",
    LAC_E_CAPACITY: "LAC_E_CAPACITY", LAC_E_HIP: "LAC_E_HIP", LAC_E_STATE: "LAC_E_STATE",
    LAC_E_FLUSH_ZERO_WIDTH: "LAC_E_FLUSH_ZERO_WIDTH", LAC_E_FLUSH_LOOP: "LAC_E_FLUSH_LOOP",
    LAC_E_UNDETERMINED: "LAC_E_UNDETERMINED",
}

# (name, restype, argtypes) for every symbol include/lac.h declares
_vp, _i, _i64, _u64 = C.c_void_p, C.c_int, C.c_int64, C.c_uint64
PROTOTYPES = [
    ("lac_version", C.c_char_p, []),
    ("lac_last_error", C.c_char_p, []),
    ("lac_open", _i, [_i, _i, _i64, _i64, _i, _u64, C.POINTER(_vp)]),
    ("lac_close", _i, [_vp]),
    ("lac_encode_reset", _i, [_vp, _vp]),
    ("lac_encode", _i, [_vp, _vp, _i64, _i64, _vp, _i64, _vp, _vp]),
    ("lac_encode_job", _i, [_vp, _vp, _i64, _i64, _vp, _i64, _vp, _vp]),
    ("lac_set_option", _i, [_vp, _i, _i64]),
    ("lac_encode_finish", _i, [_vp, _vp]),
    ("lac_encode_rebase", _i, [_vp, _vp]),
    ("lac_stream_status", _i, [_vp, _vp, _vp, _vp]),
    ("lac_encoded_lengths", _i, [_vp, _vp, _vp]),
    ("lac_encoded_device", _i, [_vp, C.POINTER(_vp), C.POINTER(_u64), C.POINTER(_vp)]),
    ("lac_copy_bits", _i, [_vp, _vp, _u64, _vp]),
    ("lac_copy_bits_dev", _i, [_vp, _vp, _u64, _vp]),
    ("lac_copy_nbits_dev", _i, [_vp, _vp, _vp]),
    ("lac_pack_bits", _i, [_vp, _vp, C.c_int, _vp, _vp]),
    ("lac_pack_bits_at", _i, [_vp, _vp, _u64, C.c_int, _vp, _vp, _vp, _vp]),
    ("lac_pack_jobs", _i, [C.c_int, _vp, _u64, _vp, _i64, _i64, _u64, _vp, _u64, C.c_int, _vp, _vp, _vp, _vp]),
    ("lac_set_output", _i, [_vp, _vp, _vp]),
    ("lac_host_alloc", _i, [_u64, C.POINTER(_vp), C.POINTER(_vp)]),
    ("lac_host_free", _i, [_vp]),
    ("lac_encode_get_state", _i, [_vp, _vp, _vp, _vp]),
    ("lac_encode_set_state", _i, [_vp, _vp, _vp, _vp]),
    ("lac_flush_digits", _i, [_vp, _vp, _vp, _vp]),
    ("lac_encoder_registers", _i, [_vp, _vp, _vp, _vp]),
    ("lac_decode_open", _i, [_vp, _vp, _u64, _vp, _vp]),
    ("lac_decode_step", _i, [_vp, _vp, _i64, _vp, _vp]),
    ("lac_decode_steps", _i, [_vp, _vp, _i64, _i64, _i64, _vp, _vp]),
    ("lac_decode_determined", _i, [_vp, _vp, _vp]),
    ("lac_decode_get_state", _i, [_vp, _vp, _vp]),
    ("lac_decode_set_state", _i, [_vp, _vp, _vp]),
    ("lac_decode_tail_begin", _i, [_vp, _vp]),
    ("lac_decode_tail_step", _i, [_vp, _vp, _i64, _i, _vp, _vp, _vp]),
    ("lac_decode_tail_get_state", _i, [_vp, _vp, _vp]),
    ("lac_decode_tail_set_state", _i, [_vp, _vp, _vp]),
    ("lac_hc_encode_symbol", _i, [_i, _vp, _vp, _i64, _i64, _vp, _vp]),
    ("lac_hc_encode_flush", _i, [_i, _i64, _i64, _vp, _vp]),
    ("lac_hc_decode_emit", _i, [_i, _vp, _i64, _i64, _i]),
    ("lac_q1_group_aborted", _i, [_vp, _vp, _vp]),
    ("lac_profile_enable", _i, [_vp, _i]),
    ("lac_profile_read", _i, [_vp, _vp, _vp, _i]),
    ("lac_q1_k", _i, [_i, _i64]),
    ("lac_encode_logits_job", _i, [_vp, _vp, _i, _i64, _i64, _vp, _i64, _vp, _vp]),
    ("lac_encode_logits", _i, [_vp, _vp, _i, _i64, _i64, _vp, _i64, _vp, _vp]),
    ("lac_decode_logits_steps", _i, [_vp, _vp, _i, _i64, _i64, _i64, _vp, _vp]),
    ("lac_quantize_logits", _i, [_vp, _vp, _i, _i64, _i64, _i64, _vp, _vp]),
]

KERNEL_IDS = {"row_stats": 0, "encode": 1, "finish": 2, "decode_step": 3, "encode_fused": 4, "decode_wave": 5,
              "q1_stats": 6, "q1_decode": 7}
LAC_LOGITS_BF16, LAC_LOGITS_F32 = 1, 2
LAC_OPT_ENCODE_PATH = 1
LAC_OPT_FUSED_MIN_STREAMS = 2
LAC_PATH_AUTO, LAC_PATH_SPLIT, LAC_PATH_FUSED, LAC_PATH_STATS, LAC_PATH_BLOCK = 0, 1, 2, 3, 4
LAC_OPT_MAPPING = 3
LAC_OPT_TERMINATION = 4
LAC_OPT_DECODE_PATH = 5
LAC_OPT_Q1_SHAPE = 6
LAC_OPT_DECODE_FINE = 7
LAC_OPT_BLOCK_WAVES = 8
LAC_OPT_DECODE_STOP = 9
LAC_MAP_CEIL, LAC_MAP_FLOOR = 0, 1
LAC_TERM_FLUSH, LAC_TERM_ACSAMPLER = 0, 1
LAC_TAIL_DECIDE, LAC_TAIL_FLUSH = 0, 1


class LacLibraryError(RuntimeError):
    pass


class LacError(RuntimeError):
    def __init__(self, code, msg=""):
        super().__init__(f"{STATUS_NAMES.get(code, code)}: {msg}")
        self.code = code


_lib = None


def load():
    """Load liblac.so (once).  Raises LacLibraryError if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise LacLibraryError(f"{LIB_PATH} is missing: build it with `python -m lac_amd.build` "
                              "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    try:
        lib = C.CDLL(LIB_PATH)
    except OSError as e:
        raise LacLibraryError(f"cannot load {LIB_PATH}: {e}") from e
    for name, res, args in PROTOTYPES:
        try:
            f = getattr(lib, name)
        except AttributeError:
            if os.environ.get("LAC_LIB"):      # an older tuning variant (A/B runs): newer entry points absent
                continue
            raise LacLibraryError(f"{LIB_PATH} lacks {name}: rebuild it (python -m lac_amd.build)") from None
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def check(rc):
    if rc != LAC_OK:
        raise LacError(rc, load().lac_last_error().decode(errors="replace"))
    return rc
