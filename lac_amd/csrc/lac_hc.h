// lac_hc.h -- host-side register arithmetic for predictors with their own mapping
// (include/lac.h "predictor-mapped coding", lac_amd/mapped.py): the coder's
// narrowing, decide_bit / emit_bit loop, flush and emit_symbol overlap check of
// /root/reference/arith_code.py:169-202, 274-291, on signed 64-bit registers kept
// within +-2^62.  Every product and doubling is formed in 128 bits and narrowed
// only after the range check, so no input -- prec up to 61, registers up to
// +-2^62, any int64 range -- overflows (checked under UBSan by tests/native).
// Shared by liblac.so (lac_api.hip wraps each in its C-ABI entry point) and
// the host sanitizer build.  No device code.
#pragma once

#include <stdint.h>

#include "lac.h"
#include "lac_core.h"

namespace lac {
namespace hc {

inline bool regs_ok(int64_t a, int64_t b) {
    const int64_t lim = (int64_t)1 << 62;
    return a > -lim && a < lim && b > -lim && b < lim;
}

// One emit_bit step (arith_code.py:181-184) l' = 2l - dD, h' = 2h + 1 - dD in 128
// bits, narrowed only when both stay within +-2^62: at prec 60-61 with |d| >= 2, or
// with l near 2^62, the 64-bit form overflows.
inline bool emit(int64_t &l, int64_t &h, int64_t d, int64_t D) {
    const i128 nl = (i128)l * 2 - (i128)d * D, nh = (i128)h * 2 + 1 - (i128)d * D;
    if (nl != (i128)(int64_t)nl || nh != (i128)(int64_t)nh || !regs_ok((int64_t)nl, (int64_t)nh)) return false;
    l = (int64_t)nl;
    h = (int64_t)nh;
    return true;
}

// closed intervals [a, b] and [c, e] in 128 bits: max(0, min(e, b) - max(a, c) + 1)
// (region_overlap, arith_code.py:59-61)
inline i128 overlap128(i128 a, i128 b, i128 c, i128 e) {
    const i128 r = (e < b ? e : b) - (a > c ? a : c) + 1;
    return r > 0 ? r : 0;
}

// receive_symbol's narrowing to [l + lo, l + hi - 1] plus the decide_bit / emit_bit
// loop (arith_code.py:169-186): the digits emitted.
inline int encode_symbol(int prec, int64_t *l, int64_t *h, int64_t lo, int64_t hi, int8_t *digits, int32_t *ndigits,
                         const char **msg) {
    if (!l || !h || !digits || !ndigits) return *msg = "NULL argument", LAC_E_ARG;
    if (prec < 2 || prec > 61) return *msg = "prec outside [2, 61]", LAC_E_PREC;
    *ndigits = 0;
    if (hi <= lo) return *msg = "empty symbol range: the reference loops forever", LAC_E_ZERO_WIDTH;
    if (!regs_ok(*l, *h)) return *msg = "registers beyond +-2^62", LAC_E_ARG;
    const int64_t D = (int64_t)1 << prec, H = D >> 1;
    const i128 nl = (i128)*l + lo, nh = (i128)*l + hi - 1;
    if (nl != (i128)(int64_t)nl || nh != (i128)(int64_t)nh || !regs_ok((int64_t)nl, (int64_t)nh))
        return *msg = "range moves the registers beyond +-2^62", LAC_E_ARG;
    int64_t L = (int64_t)nl, Hh = (int64_t)nh;
    int n = 0;
    while ((i128)Hh - L < H) {                             // decide_bit / emit_bit, arith_code.py:176-186
        const int64_t d = floordiv_pos(L, H);
        if (n >= 64 || d < -128 || d > 127) return *msg = "renormalisation out of range", LAC_E_ARG;
        digits[n++] = (int8_t)d;
        if (!emit(L, Hh, d, D)) return *msg = "registers beyond +-2^62", LAC_E_ARG;
    }
    *l = L;
    *h = Hh;
    *ndigits = n;
    return LAC_OK;
}

// A_to_bin.flush (arith_code.py:193-202): its digits.
inline int encode_flush(int prec, int64_t l, int64_t h, int8_t *digits, int32_t *ndigits, const char **msg) {
    if (!digits || !ndigits) return *msg = "NULL argument", LAC_E_ARG;
    if (prec < 2 || prec > 61) return *msg = "prec outside [2, 61]", LAC_E_PREC;
    if (!regs_ok(l, h)) return *msg = "registers beyond +-2^62", LAC_E_ARG;
    const int64_t D = (int64_t)1 << prec, Hd = D >> 1;
    int n = 0;
    *ndigits = 0;
    while (l > 0 || (i128)h + 1 < D) {                     // A_to_bin.flush, arith_code.py:193-202
        int64_t d = floordiv_pos(l, Hd);
        if (overlap128(l, h, (i128)d * Hd, (i128)(d + 1) * Hd) < overlap128(l, h, (i128)(d + 1) * Hd, (i128)(d + 2) * Hd))
            d += 1;
        if (n >= 64 || d < -128 || d > 127) return *msg = "flush out of range", LAC_E_ARG;
        digits[n++] = (int8_t)d;
        if (!emit(l, h, d, D)) return *msg = "registers beyond +-2^62", LAC_E_ARG;
    }
    *ndigits = n;
    return LAC_OK;
}

// emit_symbol (arith_code.py:274-283) on regs = {l, h, lb, hb}: the range must meet
// the received window; then, if renormalise, the emit_bit loop (:284-291).
inline int decode_emit(int prec, int64_t *regs, int64_t lo, int64_t hi, int renormalise, const char **msg) {
    if (!regs) return *msg = "NULL argument", LAC_E_ARG;
    if (prec < 2 || prec > 61) return *msg = "prec outside [2, 61]", LAC_E_PREC;
    int64_t l = regs[0], h = regs[1], lb = regs[2], hb = regs[3];
    if (!regs_ok(l, h) || !regs_ok(lb, hb)) return *msg = "registers beyond +-2^62", LAC_E_ARG;
    const i128 nl = (i128)l + lo, nh = (i128)l + hi - 1;
    if (overlap128(nl, nh, lb, hb) == 0) return *msg = "predictor range does not correspond to val", LAC_E_DECODE_RANGE;
    if (nl != (i128)(int64_t)nl || nh != (i128)(int64_t)nh || !regs_ok((int64_t)nl, (int64_t)nh))
        return *msg = "range moves the registers beyond +-2^62", LAC_E_ARG;
    l = (int64_t)nl;
    h = (int64_t)nh;
    const int64_t D = (int64_t)1 << prec, H = D >> 1;
    int n = 0;
    while (renormalise && (i128)h - l < H) {               // emit_bit, :284-291
        const int64_t d = floordiv_pos(l, H);
        if (++n > 128 || !emit(l, h, d, D) || !emit(lb, hb, d, D)) return *msg = "registers out of range", LAC_E_ARG;
    }
    regs[0] = l;
    regs[1] = h;
    regs[2] = lb;
    regs[3] = hb;
    return LAC_OK;
}

}  // namespace hc
}  // namespace lac
