// Host-side unit check of lac_amd/csrc/lac_core.h -- test infrastructure.
//
// Drives the same per-stream arithmetic the gfx950 kernels use (closed-form fudge,
// float64-assisted exact division, O(1) renorm, A/C bit planes, backward carry
// resolution) sequentially on the CPU, so tests can compare it with the oracle
// before any GPU is involved.  The wave-parallel parts (row scans, chunk search)
// are exercised only by the GPU parity tests.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <vector>

#include "lac_core.h"
#include "lac_hc.h"

using namespace lac;

extern "C" {

// the predictor-mapped host register functions (lac_hc.h, liblac's lac_hc_*)
int cc_hc_encode_symbol(int prec, int64_t *l, int64_t *h, int64_t lo, int64_t hi, int8_t *digits, int32_t *n) {
    const char *m = "";
    return hc::encode_symbol(prec, l, h, lo, hi, digits, n, &m);
}
int cc_hc_encode_flush(int prec, int64_t l, int64_t h, int8_t *digits, int32_t *n) {
    const char *m = "";
    return hc::encode_flush(prec, l, h, digits, n, &m);
}
int cc_hc_decode_emit(int prec, int64_t *regs, int64_t lo, int64_t hi, int renormalise) {
    const char *m = "";
    return hc::decode_emit(prec, regs, lo, hi, renormalise, &m);
}

uint64_t cc_div_floor(uint64_t nh, uint64_t nl, uint64_t d) { return div_floor(((u128)nh << 64) | nl, d); }
uint64_t cc_div_floor_inv(uint64_t nh, uint64_t nl, uint64_t d) {
    return div_floor_inv(((u128)nh << 64) | nl, d, 1.0 / (double)d);
}

// div_floor_inv with the reciprocal moved `ulps` ULPs off the correctly rounded
// 1/d (the device's v_rcp_f64 is an approximation); *fixups = final corrections.
uint64_t cc_div_floor_inv_ulp(uint64_t nh, uint64_t nl, uint64_t d, int ulps, int *fixups) {
    double inv = 1.0 / (double)d;
    for (int i = 0; i < (ulps < 0 ? -ulps : ulps); i++) inv = nextafter(inv, ulps < 0 ? 0.0 : 1.0e300);
    *fixups = 0;
    return div_floor_inv_n(((u128)nh << 64) | nl, d, inv, fixups);
}

// Python's a / b for 0 <= a <= b < 2^63 (lac_core.h cr_ratio), as its bit pattern.
uint64_t cc_cr_ratio(uint64_t a, uint64_t b) {
    const double r = cr_ratio(a, b);
    uint64_t u;
    memcpy(&u, &r, 8);
    return u;
}

// floor/ceil(c*w/T) through the row fraction (~0 for rows without one).
// div_small with the reciprocal `rel` (relative) off the correctly rounded 1/d, as
// the device's v_rcp_f64 + Newton can be
uint64_t cc_div_small(uint64_t n, uint64_t m, uint64_t add, uint64_t d, double rel) {
    return div_small(n, m, add, d, (1.0 / (double)d) * (1.0 + rel));
}
// the same quotient with the decoders' branch-free correction (div_small_fix_mask)
uint64_t cc_div_small_mask(uint64_t n, uint64_t m, uint64_t add, uint64_t d, double rel) {
    return div_small_fix_mask(div_small_est(n, m, add, (1.0 / (double)d) * (1.0 + rel)), n, m, add, d);
}

// div_mid (the lean decode step's u64 ranges): one estimate with the correctly rounded 1/d
uint64_t cc_div_mid(uint64_t n, uint64_t m, uint64_t add, uint64_t d) {
    const double inv = 1.0 / (double)d;
    return div_mid_fix(div_mid_est(n, m, add, inv), n, m, add, d);
}

// div_mid_est_w (the lean step's wide ranges): the addend passed as a double
uint64_t cc_div_mid_w(uint64_t n, uint64_t m, uint64_t add, double addd, uint64_t d) {
    const double inv = 1.0 / (double)d;
    return div_mid_fix(div_mid_est_w(n, m, addd, inv), n, m, add, d);
}

// div_near (the lean decode step's u32 rows): estimate with 1/d moved `ulps` ULPs off the
// correctly rounded value (the target's device reciprocal), two sign tests; n32: n < 2^32
uint64_t cc_div_near(uint64_t n, uint64_t m, uint64_t add, uint64_t d, int ulps, int n32) {
    double inv = 1.0 / (double)d;
    for (int i = 0; i < (ulps < 0 ? -ulps : ulps); i++) inv = nextafter(inv, ulps < 0 ? 0.0 : 1.0e300);
    const uint64_t q = div_small_est(n, m, add, inv);
    return n32 ? div_near_fix<true>(q, n, m, add, d) : div_near_fix<false>(q, n, m, add, d);
}

uint64_t cc_frac_mul_div(uint64_t c, uint64_t w, uint64_t T, int ceil) {
    const uint64_t f = row_frac(c, T);
    return f == kNoFrac ? ~0ull : frac_mul_div(f, c, w, T, ceil != 0);
}
// the compare-free form of k_encode's uniform chain (T < 2^62)
uint64_t cc_frac_mul_div_uni(uint64_t c, uint64_t w, uint64_t T, int ceil) {
    const uint64_t f = row_frac(c, T);
    return f == kNoFrac || (T >> 62) ? ~0ull : frac_mul_div<true>(f, c, w, T, ceil != 0);
}
// its 32-bit-count form (k_encode's straight block; c <= T < 2^32)
uint64_t cc_frac_mul_div32(uint64_t c, uint64_t w, uint64_t T, int ceil) {
    const uint64_t f = row_frac(c, T);
    if (f == kNoFrac || (T >> 32) || c > T) return ~0ull;
    return ceil ? frac_mul_div32<true>(f, (uint32_t)c, w, (uint32_t)T)
                : frac_mul_div32<false>(f, (uint32_t)c, w, (uint32_t)T);
}

// pmf rows [steps][V] (eb = 4 or 8 bytes), one stream.  Returns status, writes
// MSB-first bytes and the bit count.
int cc_encode(const void *pmf, int eb, int64_t V, int64_t steps, int64_t step_stride, const int32_t *syms, int prec,
              uint8_t *out, uint64_t cap_bytes, uint64_t *nbits) {
    const uint64_t cap_words = cap_bytes / 8;
    std::vector<uint64_t> A(cap_words + 1, 0), Cc(cap_words + 1, 0);
    int64_t l = 0, h = ((int64_t)1 << prec) - 1;
    uint64_t L = 0, wa = 0, wc = 0;
    auto store = [&](uint64_t idx, uint64_t a, uint64_t c) { A[idx] = a; Cc[idx] = c; };
    for (int64_t t = 0; t < steps; t++) {
        const char *row = (const char *)pmf + (size_t)(t * step_stride) * eb;
        auto at = [&](int64_t i) -> uint64_t { return eb == 4 ? ((const uint32_t *)row)[i] : ((const uint64_t *)row)[i]; };
        const int64_t s = syms[t];
        if (s < 0 || s >= V) return -3;
        u128 T = 0, lo = 0;
        uint64_t minp = 0;
        for (int64_t i = 0; i < V; i++) {
            const uint64_t p = at(i);
            if (i < s) lo += p;
            T += p;
            if (p && (!minp || p < minp)) minp = p;
        }
        if (T == 0 || (T >> 64)) return -5;
        const uint64_t hi = (uint64_t)lo + at(s);
        const uint64_t w = (uint64_t)(h - l + 1);
        uint64_t a, b;
        const uint64_t flo = row_frac((uint64_t)lo, (uint64_t)T), fhi = row_frac(hi, (uint64_t)T);
        if (!is_fudged((uint64_t)T, w, minp) && flo != kNoFrac) {         // k_encode's split-path form
            a = frac_mul_div(flo, (uint64_t)lo, w, (uint64_t)T, true);
            b = frac_mul_div(fhi, hi, w, (uint64_t)T, true);
        } else if (!is_fudged((uint64_t)T, w, minp)) {
            unfudged_range((uint64_t)lo, hi, (uint64_t)T, w, &a, &b);
        } else {
            i128 xprev = (i128)((u128)1 << 127);
            uint64_t c = 0;
            for (int64_t j = 0; j < s; j++) {
                c += at(j);
                const i128 X = fudge_x(c, j, w, (uint64_t)T);
                if (X > xprev) xprev = X;
            }
            const i128 xs = fudge_x(hi, s, w, (uint64_t)T);
            a = s > 0 ? fudge_f(s - 1, xprev, (uint64_t)T, w, V) : 0;
            b = fudge_f(s, xs > xprev ? xs : xprev, (uint64_t)T, w, V);
        }
        if (a >= b) return -4;
        h = l + (int64_t)b - 1;
        l = l + (int64_t)a;
        int k;
        uint64_t E;
        renorm(l, h, prec, &k, &E);
        if (!plane_append(L, wa, wc, k, E, cap_words, store)) return -7;
    }
    if (L > 0) { A[(L - 1) >> 6] = wa; Cc[(L - 1) >> 6] = wc; }
    int8_t fd[8];
    const int m = flush_digits(l, h, prec, fd);
    if (m < 0) return -7;
    int64_t F = 0;
    for (int i = 0; i < m; i++) F = F * 2 + fd[i];
    const uint64_t Lf = L + (uint64_t)m, nwords = (Lf + 63) >> 6;
    if (nwords > cap_words) return -7;
    const int pad = (int)(nwords * 64 - Lf);
    i128 carry = (i128)F * ((i128)1 << pad);
    const int64_t last = L ? (int64_t)((L - 1) >> 6) : -1;
    for (int64_t i = (int64_t)nwords - 1; i >= 0; i--) {
        const uint64_t av = i <= last ? A[i] : 0, cv = i <= last ? Cc[i] : 0;
        const i128 sm = (i128)(u128)av + (i128)(u128)cv + carry;
        const uint64_t o = bswap64((uint64_t)sm);
        memcpy(out + 8 * i, &o, 8);
        carry = sm >> 64;
    }
    if (carry != 0) return -1;
    *nbits = Lf;
    return 0;
}

}  // extern "C"
