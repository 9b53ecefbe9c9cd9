// lac_core.h -- per-stream coder arithmetic for gfx950 (host-callable for unit checks).
//
// Everything here is exact integer arithmetic restating /root/reference/arith_code.py:
//
//  * ceil mapping of CDFPredictor.symbol_to_range (:98-110):
//        a = ceil(lo*w/T), b = ceil(hi*w/T)            -> unfudged_range()
//  * the fudge branch of CDFPredictor.fudged_dist (:83-93) in closed form.  The
//    loop p_i = max(p_{i-1}+1, min(w-(V-1-i), floor(c_i*w/T))) equals
//        f_i = i + max(1, min(w-V+1, floor(Xmax_i / T))),
//        Xmax_i = max_{j<=i} (c_j*w - j*T)
//    so a = f_{s-1}, b = f_s need one prefix max and one division   -> fudge_f()
//  * decide_bit/emit_bit (:176-186) collapsed: the loop runs
//        k = max(0, prec - bitlen(h-l))
//    times and emits digits whose value as one integer is E = l >> (prec-k);
//    then l' = (l mod 2^(prec-k)) << k, h' = l' + ((h-l+1) << k) - 1  -> renorm()
//  * flush (:193-202) literally, with region_overlap (:59-61)          -> flush_digits()
//
// The output integer R = sum_k d_k 2^(L-1-k) (A_to_bin.encode :212-219 == bits())
// is accumulated as two bit planes: A (the low k bits of each E, appended) and C
// (E's carry bit, which lands on the last bit already written).  R = A + C + flush,
// resolved by one backward big-integer add in the finish kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#ifndef LAC_PLANE_FAST
#define LAC_PLANE_FAST 1     // plane_append: the within-one-word case without the loop
#endif
#ifndef LAC_ENC_STRAIGHT
#define LAC_ENC_STRAIGHT 1   // k_encode: 64-step blocks without per-step tests where no step can need one
#endif
#ifndef LAC_ENC_PIPE
#define LAC_ENC_PIPE 1       // k_encode straight blocks: the next step's row values read one step ahead
#endif
#ifndef LAC_ENC_UNROLL
#define LAC_ENC_UNROLL 2     // k_encode straight blocks: steps per loop iteration
#endif

namespace lac {

typedef unsigned __int128 u128;
typedef __int128 i128;

struct RowStats {          // per (step, stream) row, written by the row-stats kernel
    uint64_t lo;           // c_{s-1} = sum_{i<s} pmf_i
    uint64_t hi;           // c_s
    uint64_t tot;          // T = c_{V-1}; 0 marks a bad row (minp: 0 empty, 1 overflow)
    uint64_t minp;         // smallest positive pmf entry
    double inv_tot;        // 1.0 / T, so the serial coder step multiplies instead of divides
    uint64_t pad;
};

struct EncState {          // per stream, persistent across lac_encode calls
    int64_t l, h;          // coder registers, 0 <= l < 2^(prec+1), h < 3*2^prec
    uint64_t L;            // bits written to the planes so far
    uint64_t wa, wc;       // plane words holding bit L-1 (not yet stored)
    int64_t nsym;          // symbols encoded
    int32_t err;           // sticky status (LAC_E_*)
    int32_t nflush;        // flush digits (finish)
    int64_t err_step;      // nsym at the failing symbol
    int8_t flush[8];       // flush digits
};

struct TailState {                 // the decoder's tail in the reference frame; mirrors lac_tail_state (include/lac.h)
    int64_t l, h, lb, hb;
    int32_t err, done;
    int64_t still, nsym;
};

struct DecState {
    int64_t l, h, x;       // registers and the prec-bit value window (bits past the end read as 0)
    uint64_t pos;          // next bit to read
    int64_t nsym;
    int32_t err;
    int32_t det;           // 1 while every symbol so far was determined by the available bits
    int64_t err_step;
    int64_t ndet;          // leading symbols A_from_bin.run(bits, stop=0) emits (arith_code.py:268-299)
};

__host__ __device__ inline int bitlen64(uint64_t x) { return x ? 64 - __builtin_clzll(x) : 0; }

__host__ __device__ inline uint64_t div_floor_inv(u128 N, uint64_t d, double inv);

// The first quotient estimate of div_floor / div_floor_inv is a double; one at or
// above 2^64 (a quotient near 2^64 - 1, estimated high) starts from the largest
// double below 2^64 instead, so the estimate stays within a few thousand of the
// quotient and the second estimate leaves at most two +-1 corrections
// (tests/test_core_host.py, also with the reciprocal 4 ULPs off).
constexpr uint64_t kTopQ = 0xFFFFFFFFFFFFF800ull;

// A remainder as a double: one rounding when it fits 64 bits (the split form
// below rounds the low word of a small negative remainder to a multiple of 2^11,
// which cost up to ~1024/d final corrections).
__host__ __device__ inline double i128_to_double(i128 r) {
    const int64_t lo = (int64_t)(uint64_t)r;
    if ((i128)lo == r) return (double)lo;
    return (double)(int64_t)(r >> 64) * 18446744073709551616.0 + (double)(uint64_t)r;
}

// 1/d for the quotient estimates of div_floor_inv.  On the device v_rcp_f64 plus
// one Newton step (no IEEE divide sequence on the coder's latency chain).
// v_rcp_f64 alone is good to only ~2^-25 relative (measured on the MI355X: up to
// 2.6e8 ULPs, tools/rcp_probe.hip, profiles/r03/rcp_probe_before.json): the
// second estimate of a quotient near 2^60 was then still ~2^10 off, and the +-1
// correction loop of div_floor_inv ran up to 35 000 times (u64-table decode
// targets).  The Newton step squares the error (two FMAs); results were exact
// either way.
__host__ __device__ inline double recip(uint64_t d) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double dd = (double)d;
    const double r = __builtin_amdgcn_rcp(dd);
    return __builtin_fma(r, __builtin_fma(-dd, r, 1.0), r);
#else
    return 1.0 / (double)d;
#endif
}

// floor(N / d) for d > 0 when the quotient is known to be < 2^64 (the decode target
// floor(v*T/w) reaches 2^64 - 1 for u64 tables with totals near 2^64).  Two rounds of
// float64 quotient estimates plus an exact 128-bit remainder correction: no
// shift-subtract loop (the generic __int128 division is ~5k cycles on gfx950).
__host__ __device__ inline uint64_t div_floor(u128 N, uint64_t d) {
#if defined(__HIP_DEVICE_COMPILE__)
    return div_floor_inv(N, d, recip(d));
#endif
    const double two64 = 18446744073709551616.0;
    const double dd = (double)d;
    const double dn = (double)(uint64_t)(N >> 64) * two64 + (double)(uint64_t)N;
    double qd = dn / dd;
    uint64_t q = qd >= two64 ? kTopQ : (uint64_t)qd;
    i128 r = (i128)(N - (u128)q * d);
    const double rd = i128_to_double(r);
    const int64_t adj = (int64_t)(rd / dd);
    q += (uint64_t)adj;
    r -= (i128)adj * (i128)d;
    while (r < 0) { q -= 1; r += d; }
    while (r >= (i128)d) { q += 1; r -= d; }
    return q;
}

__host__ __device__ inline uint64_t div_ceil(u128 N, uint64_t d) {
    return div_floor(N + (d - 1), d);
}

// div_floor with a precomputed inv = 1.0 / d (same estimate accuracy, no
// float64 divide on the latency chain of the sequential coder).  `fixups`, when
// not null, counts the final +-1 corrections (host checks bound them for an
// inv off the correctly rounded 1/d by the device reciprocal's error).
__host__ __device__ inline uint64_t div_floor_inv_n(u128 N, uint64_t d, double inv, int *fixups) {
    const double two64 = 18446744073709551616.0;
    const double dn = (double)(uint64_t)(N >> 64) * two64 + (double)(uint64_t)N;
    double qd = dn * inv;
    uint64_t q = qd >= two64 ? kTopQ : (uint64_t)qd;
    i128 r = (i128)(N - (u128)q * d);
    const double rd = i128_to_double(r);
    const int64_t adj = (int64_t)(rd * inv);
    q += (uint64_t)adj;
    r -= (i128)adj * (i128)d;
    while (r < 0) { q -= 1; r += d; if (fixups) ++*fixups; }
    while (r >= (i128)d) { q += 1; r -= d; if (fixups) ++*fixups; }
    return q;
}
__host__ __device__ inline uint64_t div_floor_inv(u128 N, uint64_t d, double inv) {
    return div_floor_inv_n(N, d, inv, nullptr);
}

// Exact conversions between integers below 2^52 and doubles by the 2^52 magic: the
// integer as the mantissa of a double of exponent 52 (one OR and one subtract, where a
// general u64 <-> f64 conversion is four or six operations on the vector unit).
constexpr double kTwo52 = 4503599627370496.0;
__host__ __device__ inline double small_to_f64(uint64_t n) {          // n < 2^52
    const uint64_t b = 0x4330000000000000ull | n;
    double d;
    memcpy(&d, &b, 8);
    return d - kTwo52;
}
__host__ __device__ inline uint64_t f64_to_small(double e) {          // nearest integer, 0 <= e < 2^52
    const double d = e + kTwo52;
    uint64_t b;
    memcpy(&b, &d, 8);
    return b & 0x000FFFFFFFFFFFFFull;
}

// floor((n*m + add) / d) when the quotient is below 2^50 and n, m, add < 2^52 (the
// decoder's targets floor(v*T/w) and ranges ceil(c*w/T) at prec <= 50 with totals
// below 2^50): one fused double estimate, fma(n, m, add) * inv rounded to the nearest
// integer, is within q * (2^-52 + err(inv)) + 1/2 of the quotient -- under 2 for an
// inv good to 2^-50 (the device reciprocal after its Newton step) -- so the remainder
// n*m + add - q*d lies in (-3d, 3d) and wrapping 64-bit arithmetic holds it exactly;
// at most two corrections follow.  No 128-bit products: the decode step's chain of
// quarter-rate multiplies (div_floor_inv: two estimates and 128-bit remainders)
// becomes one FMA, one multiply and a 64-bit remainder.
constexpr uint64_t kSmallQuot = 1ull << 50;
__host__ __device__ inline uint64_t div_small_est(uint64_t n, uint64_t m, uint64_t add, double inv) {
    const double e = __builtin_fma(small_to_f64(n), small_to_f64(m), small_to_f64(add)) * inv;
    return f64_to_small(e > 0.0 ? e : 0.0);
}
__host__ __device__ inline uint64_t div_small_fix(uint64_t q, uint64_t n, uint64_t m, uint64_t add, uint64_t d) {
    int64_t r = (int64_t)(n * m + add - q * d);
    while (r < 0) { q -= 1; r += (int64_t)d; }
    while (r >= (int64_t)d) { q += 1; r -= (int64_t)d; }
    return q;
}
__host__ __device__ inline uint64_t div_small(uint64_t n, uint64_t m, uint64_t add, uint64_t d, double inv) {
    return div_small_fix(div_small_est(n, m, add, inv), n, m, add, d);
}
// div_small_fix without a branch, for the sequential decoders' wave-uniform chains:
// with the remainder r in [-3d, 3d) (above: the rounded estimate is at most 3 above the
// floor and 2 below it), the quotient is q - [r < -2d] - [r < -d] - [r < 0] + [r >= d] +
// [r >= 2d], each bracket the sign mask of a difference (an arithmetic shift; 0 or -1) --
// scalar adds and shifts on the GPU, where the loops' ordered 64-bit tests were VALU
// compares feeding a branch each.
__host__ __device__ inline uint64_t sign_mask64(uint64_t x) { return (uint64_t)((int64_t)x >> 63); }
__host__ __device__ inline uint64_t div_small_fix_mask(uint64_t q, uint64_t n, uint64_t m, uint64_t add, uint64_t d) {
    const uint64_t r = n * m + add - q * d;
    return q + 2 + sign_mask64(r + 2 * d) + sign_mask64(r + d) + sign_mask64(r) + sign_mask64(r - d) +
           sign_mask64(r - 2 * d);
}

// floor((n*m + add) / d) for a quotient of at most 2^50 with any d < 2^64, n < 2^64,
// m <= 2^51, add < d (the lean decode step's ranges ceil(c*w/T) on u64 rows with totals
// of 2^50 and more, prec <= 50 so w <= 2^50, where div_small's 64-bit remainder no longer
// holds the error).  One double estimate, fma(n, m, add) * inv with inv the correctly
// rounded 1/d: a few ulps of relative error, within 1/2 of the quotient, so its floor is
// the quotient or one off either way; the 128-bit remainder N - q*d, in [-d, 2d), then
// decides the correction by its sign and size, without branches.
__host__ __device__ inline uint64_t div_mid_est(uint64_t n, uint64_t m, uint64_t add, double inv) {
    const double e = __builtin_fma((double)n, (double)m, (double)add) * inv;
    return (uint64_t)(e > 0.0 ? e : 0.0);
}
// div_mid_est for the lean step's wide ranges, in fewer conversions: m below 2^52 through the
// 2^52 magic, the addend given as a double (the ceil mapping's T - 1 as T rounded to a double,
// which moves the quotient by under 2^-38 for T >= 2^50), and the estimate rounded to the
// nearest integer by the magic (quotients <= 2^50).  Within one of the quotient, as
// div_mid_fix takes it (host-checked, tests/test_core_host.py).
__host__ __device__ inline uint64_t div_mid_est_w(uint64_t n, uint64_t m, double addd, double inv) {
    const double e = __builtin_fma((double)n, small_to_f64(m), addd) * inv;
    return f64_to_small(e > 0.0 ? e : 0.0);
}
__host__ __device__ inline uint64_t div_mid_fix(uint64_t q, uint64_t n, uint64_t m, uint64_t add, uint64_t d) {
    const u128 r = (u128)n * m + add - (u128)q * d;          // wrapping: [-d, 2d) as two's complement
    const uint64_t rh = (uint64_t)(r >> 64), rl = (uint64_t)r;
    const uint64_t neg = rh >> 63;
    const uint64_t ge = (neg ^ 1) & ((uint64_t)(rh != 0) | (uint64_t)(rl >= d));
    return q - neg + ge;
}

// floor((n*m + add) / d) from a rounded estimate within one of the quotient (div_small_est
// with inv good to a few ulps and a quotient whose ulps stay below 1/2) and a remainder
// n*m + add - q*d in [-d, 2d) that wrapping 64-bit arithmetic holds (d < 2^62): two sign
// tests instead of div_small_fix_mask's five.  The lean decode step's u32 rows (T < 2^32):
// the target floor(v*T/w) (quotient < 2^32, inv = the device reciprocal of w) and the
// ranges ceil(c*w/T) (c <= T, quotient <= 2^50, inv = 1/T correctly rounded).  N32: n
// below 2^32 (the ranges' CDF entries), so n*m is a 32 x 64-bit product.
template <bool N32 = false>
__host__ __device__ inline uint64_t div_near_fix(uint64_t q, uint64_t n, uint64_t m, uint64_t add, uint64_t d) {
    const uint64_t nm = N32 ? (uint64_t)(uint32_t)n * m : n * m;
    const uint64_t r = nm + add - q * d;
    const uint64_t neg = sign_mask64(r);                      // r < 0: one less
    const uint64_t ge = ~sign_mask64(r - d) & ~neg;           // r >= d: one more
    return q + neg - ge;
}

// CDFPredictor.fudged_dist test (arith_code.py:84): fudged iff T > w*minp.
__host__ __device__ inline bool is_fudged(uint64_t T, uint64_t w, uint64_t minp) {
    return (u128)T > (u128)w * minp;
}

// Unfudged ceil mapping (arith_code.py:107-109).
__host__ __device__ inline void unfudged_range(uint64_t lo, uint64_t hi, uint64_t T, uint64_t w,
                                               uint64_t *a, uint64_t *b) {
    *a = lo ? div_ceil((u128)lo * w, T) : 0;
    *b = div_ceil((u128)hi * w, T);
}

__host__ __device__ inline void unfudged_range_inv(uint64_t lo, uint64_t hi, uint64_t T, double inv, uint64_t w,
                                                   uint64_t *a, uint64_t *b) {
    *a = lo ? div_floor_inv((u128)lo * w + (T - 1), T, inv) : 0;
    *b = div_floor_inv((u128)hi * w + (T - 1), T, inv);
}

// Row fractions for the sequential coder step of the split path.  For a row with
// total T < 2^63 and a cumulative count 0 <= c <= T, f = floor(c * 2^63 / T)
// (c == T gives exactly 2^63).  They depend only on the row, so k_encode computes
// them for 64 steps at once (one lane per step) and the serial step is left with
// multiplications.  kNoFrac marks rows with T >= 2^63: those divide as before.
constexpr uint64_t kNoFrac = ~0ull;
__host__ __device__ inline uint64_t row_frac(uint64_t c, uint64_t T) {
    if (T == 0 || (T >> 63)) return kNoFrac;
    if (c >= T) return 1ull << 63;
    // c < T: quotient < 2^63.  A correctly rounded 1/T (IEEE divide, not the
    // approximate v_rcp_f64 of recip()): with quotients this close to 2^63 the
    // reciprocal's error sets how many correction steps div_floor_inv loops.
    return div_floor_inv((u128)c << 63, T, 1.0 / (double)T);
}

// floor(c*w/T) (ceil when `ceil`) from f = row_frac(c, T), for w <= 2^61 (prec
// <= 61) and T < 2^63.  f*w/2^63 lies within w/2^63 <= 1/4 below c*w/T, so
// q = floor(f*w/2^63) is the floor or one less; the remainder c*w - q*T is then
// in [0, 2T), below 2^64, so wrapping 64-bit arithmetic computes it exactly.
// d >= 0 for a wave-uniform d, tested on the high word alone.  On gfx950 the compiler
// lowers every 64-bit ordered compare -- even of SGPR operands, even against 0 -- to a
// VALU v_cmp whose result crosses back to the scalar unit; an empty asm holding the high
// word in an SGPR keeps the 32-bit test (s_cmp) from being folded back into one.
// Uniform values only.
__host__ __device__ inline bool nonneg_uni(int64_t d) {
#if defined(__HIP_DEVICE_COMPILE__)
    int hi = (int)((uint64_t)d >> 32);
    asm("" : "+s"(hi));
    return hi >= 0;
#else
    return d >= 0;
#endif
}

//
// UNIF (the wave-uniform chain of k_encode; needs T < 2^62): the same quotient with no
// compare at all.  With r = c*w - q*T (+ T - 1 for ceil) in [0, 3T - 1), the result is
// q + [r >= T] (+ [r >= 2T] for ceil), each bracket 1 + the sign mask of a difference
// (an arithmetic shift): plain scalar adds and shifts on the GPU, where an ordered
// 64-bit compare is a VALU v_cmp and a compare's boolean is a lane mask whose use moves
// the sum to the vector unit.
template <bool UNIF = false>
__host__ __device__ inline uint64_t frac_mul_div(uint64_t f, uint64_t c, uint64_t w, uint64_t T, bool ceil) {
    const u128 p = (u128)f * w;
    uint64_t q = (uint64_t)(p >> 63);
    if constexpr (UNIF) {
        const uint64_t r = c * w - q * T + (ceil ? T - 1 : 0);
        q += 1 + (uint64_t)((int64_t)(r - T) >> 63);
        if (ceil) q += 1 + (uint64_t)((int64_t)(r - 2 * T) >> 63);
        return q;
    }
    uint64_t r = c * w - q * T;
    if (r >= T) { q += 1; r -= T; }
    return q + (uint64_t)(ceil && r != 0);
}

// frac_mul_div<true> for 32-bit counts and totals (c <= T < 2^32): the remainder's two
// products then take three 32-bit multiplies each instead of four (k_encode's straight
// block, u32 tables).
template <bool CEIL>
__host__ __device__ inline uint64_t frac_mul_div32(uint64_t f, uint32_t c, uint64_t w, uint32_t T) {
    uint64_t q = (uint64_t)(((u128)f * w) >> 63);
    const uint64_t T64 = T;
    const uint64_t r = (uint64_t)c * w - q * T64 + (CEIL ? T64 - 1 : 0);
    q += 1 + (uint64_t)((int64_t)(r - T64) >> 63);
    if (CEIL) q += 1 + (uint64_t)((int64_t)(r - 2 * T64) >> 63);
    return q;
}

// Floor mapping of Predictor.symbol_to_range (arith_code.py:69-70) and of
// ACSampler's Region.map/step (arithmetic_coding.py:160-168):
// a = floor(lo*w/T), b = floor(hi*w/T).  No fudge exists on these paths.
__host__ __device__ inline void floor_range(uint64_t lo, uint64_t hi, uint64_t T, uint64_t w,
                                            uint64_t *a, uint64_t *b) {
    *a = lo ? div_floor((u128)lo * w, T) : 0;
    *b = div_floor((u128)hi * w, T);
}

// X_j = c_j*w - j*T (signed), the quantity whose prefix max drives the fudge.
__host__ __device__ inline i128 fudge_x(uint64_t c, int64_t j, uint64_t w, uint64_t T) {
    return (i128)((u128)c * w) - (i128)((u128)(uint64_t)j * T);
}

// f_i = i + max(1, min(w-V+1, floor(xmax/T)))   (fudged_dist, closed form)
__host__ __device__ inline uint64_t fudge_f(int64_t i, i128 xmax, uint64_t T, uint64_t w, int64_t V) {
    const uint64_t cap = w - (uint64_t)V + 1;             // >= 2 since w > 2^(prec-1) >= V
    uint64_t g;
    if (xmax < (i128)2 * (i128)T) {
        g = 1;                                            // floor(xmax/T) <= 1
    } else {
        const uint64_t m = div_floor((u128)xmax, T);      // <= w
        g = m < cap ? m : cap;
    }
    return (uint64_t)i + g;
}

// Encoder renormalisation (decide_bit/emit_bit, arith_code.py:176-186) in O(1).
// On return *k digits were emitted with integer value *E (< 2^(k+1)).
__host__ __device__ inline void renorm(int64_t &l, int64_t &h, int prec, int *k, uint64_t *E) {
    const int kk = prec - bitlen64((uint64_t)(h - l));
    if (kk <= 0) { *k = 0; *E = 0; return; }
    const int sh = prec - kk;
    const uint64_t e = (uint64_t)l >> sh;
    const int64_t w = h - l + 1;
    l = (int64_t)(((uint64_t)l - (e << sh)) << kk);
    h = l + (w << kk) - 1;
    *k = kk;
    *E = e;
}

__host__ __device__ inline int64_t floordiv_pos(int64_t a, int64_t b) {   // Python //, b > 0
    int64_t q = a / b;
    if ((a % b) != 0 && a < 0) q -= 1;
    return q;
}

__host__ __device__ inline int64_t overlap(int64_t a, int64_t b, int64_t c, int64_t d) {
    const int64_t hi = d < b ? d : b, lo = a > c ? a : c;
    const int64_t r = hi - lo + 1;
    return r > 0 ? r : 0;
}

// Python's `a / b` for ints 0 <= a <= b, 0 < b < 2^63: the double nearest the
// exact quotient, ties to even (CPython divides ints with correct rounding).
// A_from_bin.flush ranks its candidate symbols by such quotients
// (arith_code.py:305-307, :312), so the ranking -- ties included -- needs the
// same double.  Operands below 2^53 convert exactly and the IEEE divide rounds
// correctly; larger ones take an exact integer quotient with 55-56 significant
// bits plus a sticky remainder, rounded here to 53.
__host__ __device__ inline int bitlen_u128(u128 x) {
    const uint64_t hi = (uint64_t)(x >> 64);
    return hi ? 64 + bitlen64(hi) : bitlen64((uint64_t)x);
}
__host__ __device__ inline double cr_ratio(uint64_t a, uint64_t b) {
    if (a == 0) return 0.0;
    if (a == b) return 1.0;
    if (a < (1ull << 53) && b < (1ull << 53)) return (double)a / (double)b;
    const int s = 55 + bitlen64(b) - bitlen64(a);        // quotient a*2^s/b in (2^54, 2^56)
    const u128 N = (u128)a << s;
    const u128 Q = N / b;
    const bool sticky = (N - Q * b) != 0;
    const int drop = bitlen_u128(Q) - 53;                  // 2 or 3
    uint64_t m = (uint64_t)(Q >> drop);
    const uint64_t rest = (uint64_t)Q & ((1ull << drop) - 1), half = 1ull << (drop - 1);
    if (rest > half || (rest == half && (sticky || (m & 1)))) m += 1;
    return ldexp((double)m, drop - s);                     // m <= 2^53: exact
}

// Python's a // b (floor) for a signed 128-bit numerator and b > 0.
__host__ __device__ inline i128 floordiv_i128(i128 a, uint64_t b) {
    if (a >= 0) return (i128)((u128)a / b);
    const u128 m = (u128)(-a);
    return -(i128)((m + b - 1) / b);
}

// A_to_bin.flush (arith_code.py:193-202), literal.  Returns the digit count (<= 8
// in practice: <= 2 observed), digits may be -1..3.  Returns -1 on overrun.
__host__ __device__ inline int flush_digits(int64_t l, int64_t h, int prec, int8_t *out) {
    const int64_t D = (int64_t)1 << prec, Hd = (int64_t)1 << (prec - 1);
    int n = 0;
    while (l > 0 || h + 1 < D) {
        int64_t d = floordiv_pos(l, Hd);
        if (overlap(l, h, d * Hd, (d + 1) * Hd) < overlap(l, h, (d + 1) * Hd, (d + 2) * Hd)) d += 1;
        l = l * 2 - d * D;
        h = h * 2 + 1 - d * D;
        if (n >= 8) return -1;
        out[n++] = (int8_t)d;
    }
    return n;
}

// Append one renorm's output to the planes held in registers.  `store(idx, wa, wc)`
// receives every completed word.  Returns false on capacity overflow.
template <typename Store>
__host__ __device__ inline bool plane_append(uint64_t &L, uint64_t &wa, uint64_t &wc, int k, uint64_t E,
                                             uint64_t cap_words, Store store) {
    if (k <= 0) return true;
#if LAC_PLANE_FAST
    // the common case: the digits land inside the word bit L-1 is in (no word completes,
    // so no store and no loop), the carry on that word's bit L-1.  Bit L-1 stays in the
    // same word, which is within capacity: an earlier append put it there, or a restored
    // state did (lac_encode_set_state refuses L > cap_words * 64)
    const int off0 = (int)(L & 63);
    if (off0 != 0 && k <= 64 - off0) {                    // k <= 63
        if (E >> k) wc |= 1ull << (64 - off0);
        wa |= (E & ((1ull << k) - 1)) << (64 - off0 - k);
        L += (uint64_t)k;
        return true;
    }
#endif
    const uint64_t ehi = E >> k;
    uint64_t elo = E & ((k == 64) ? ~0ull : ((1ull << k) - 1));
    if (ehi) wc |= 1ull << (63 - ((L - 1) & 63));         // carry onto bit L-1 (L >= 1 here)
    int rem = k;
    while (rem > 0) {
        if (L > 0 && (L & 63) == 0) {                     // bit L starts a new word
            const uint64_t idx = (L >> 6) - 1;
            if (idx >= cap_words) return false;
            store(idx, wa, wc);
            wa = 0;
            wc = 0;
        }
        const int off = (int)(L & 63);
        const int take = rem < 64 - off ? rem : 64 - off;
        const uint64_t chunk = (elo >> (rem - take)) & ((take == 64) ? ~0ull : ((1ull << take) - 1));
        wa |= chunk << (64 - off - take);
        L += (uint64_t)take;
        rem -= take;
    }
    return ((L - 1) >> 6) < cap_words;
}

__host__ __device__ inline uint64_t bswap64(uint64_t x) {
    return __builtin_bswap64(x);
}

}  // namespace lac
