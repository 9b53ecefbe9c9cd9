// lac_dec_dev.h -- decode building blocks shared by the pmf decoders (lac_decode.hip)
// and the logits decoder (lac_logits.hip): the bit window, the decoder state in
// SGPRs, chunk re-scan, renormalisation (decode_advance: emit_symbol + emit_bit,
// arith_code.py:274-291, value form), the small-quotient divisions and the decoder
// state initialisation.
#pragma once
#include "lac_dev.h"

namespace {

// ------------------------------------------------------------------ decode
// Bits [pos, pos+k) of a big-endian byte stream, zeros past nbits (k <= 63).
__device__ inline uint64_t read_bits(const uint8_t *bits, uint64_t nbits, uint64_t pos, int k) {
    if (k <= 0 || pos >= nbits) return 0;
    const uint64_t *wp = reinterpret_cast<const uint64_t *>(bits);
    const uint64_t wi = pos >> 6;
    const int off = (int)(pos & 63);
    uint64_t v = bswap64(wp[wi]) << off;
    if (off && (wi + 1) * 64 < nbits) v |= bswap64(wp[wi + 1]) >> (64 - off);
    v >>= (64 - k);
    if (pos + (uint64_t)k > nbits) {
        const int drop = (int)(pos + (uint64_t)k - nbits);
        v = (v >> drop) << drop;
    }
    return v;
}

// The two stream words the next renormalisation can read (bits pos .. pos+127),
// loaded at the top of a decode step so their latency hides under the search;
// window_bits then equals read_bits(bits, nbits, pos, k) for any k <= 64.
// Indices are clamped into the stream (an empty stream reads a zero word), so
// the loads are unconditional.
struct BitWin {
    uint64_t w0, w1;
};
// (not const: a const __device__ array is placed in the constant address space, and the
// select between it and a stream pointer then turned the window loads into flat loads,
// which count in both vmcnt and lgkmcnt)
__device__ uint64_t g_zero_words[1] = {0};
__device__ inline BitWin bit_window(const uint8_t *bits, uint64_t nbits, uint64_t pos) {
    const uint64_t nw = (nbits + 63) >> 6, wi = pos >> 6;
    const uint64_t *wp = nw ? reinterpret_cast<const uint64_t *>(bits) : g_zero_words;
    const uint64_t last = nw ? nw - 1 : 0;
    return BitWin{wp[wi < last ? wi : last], wp[wi + 1 < last ? wi + 1 : last]};
}
__device__ inline uint64_t window_bits(const BitWin &win, uint64_t nbits, uint64_t pos, int k) {
    if (k <= 0 || pos >= nbits) return 0;
    const int off = (int)(pos & 63);
    uint64_t v = bswap64(win.w0) << off;
    if (off && ((pos >> 6) + 1) * 64 < nbits) v |= bswap64(win.w1) >> (64 - off);
    v >>= (64 - k);
    if (pos + (uint64_t)k > nbits) {
        const int drop = (int)(pos + (uint64_t)k - nbits);
        v = (v >> drop) << drop;
    }
    return v;
}

// window_bits for 0 <= k <= 62 with no branch (the lone-wave decoder's step): the second
// word always shifted in (its bits lie past the stream's end whenever the test above
// skips it, and the end mask clears them), shifts by 64 split into two, the end mask's
// drop clamped to 63 (past the end everything is dropped: v < 2^k).
__device__ inline uint64_t window_bits_nb(const BitWin &win, uint64_t nbits, uint64_t pos, int k) {
    const int off = (int)(pos & 63);
    uint64_t v = (bswap64(win.w0) << off) | ((bswap64(win.w1) >> 1) >> (63 - off));
    v = (v >> 1) >> (63 - k);                                 // the top k bits; 0 for k = 0
    const int64_t over = (int64_t)(pos + (uint64_t)k - nbits);
    const int drop = over <= 0 ? 0 : (over > 63 ? 63 : (int)over);
    return (v >> drop) << drop;
}

// A decoder state loaded by one wave for its own stream, moved to SGPRs: the compiler
// cannot tell a value loaded from a wave-uniform address is uniform.
__device__ inline void dec_state_uniform(DecState &st) {
    st.l = (int64_t)rfl_u64((uint64_t)st.l);
    st.h = (int64_t)rfl_u64((uint64_t)st.h);
    st.x = (int64_t)rfl_u64((uint64_t)st.x);
    st.pos = rfl_u64(st.pos);
    st.nsym = (int64_t)rfl_u64((uint64_t)st.nsym);
    st.err = __builtin_amdgcn_readfirstlane(st.err);
    st.det = __builtin_amdgcn_readfirstlane(st.det);
    st.err_step = (int64_t)rfl_u64((uint64_t)st.err_step);
    st.ndet = (int64_t)rfl_u64((uint64_t)st.ndet);
}

__global__ void k_dec_init(DecState *states, int64_t B, int prec, const uint8_t *bits, uint64_t stride,
                           const uint64_t *nbits) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    DecState st;
    memset(&st, 0, sizeof(st));
    st.l = 0;
    st.h = ((int64_t)1 << prec) - 1;
    st.pos = (uint64_t)prec;
    st.err_step = -1;
    st.det = 1;
    st.ndet = 0;
    // A stream claiming more bits than its row holds would make every later
    // bit-window load run past the row (and past the buffer for the last
    // stream): it fails with a sticky LAC_E_ARG before anything is read.
    if (nbits[b] > stride * 8) {
        st.err = LAC_E_ARG;
        st.err_step = 0;
    } else {
        st.x = (int64_t)read_bits(bits + b * stride, nbits[b], 0, prec);
    }
    states[b] = st;
}

// One decode step for every stream: grid = B workgroups of 256 threads.
// ---- decode building blocks (one wave; all values wave-uniform unless noted)

// Re-scan one chunk (vectors cv0 + 64*g + lane, g < G) from cumulative base cb:
// count of entries with c_i <= tgt, and the bracketing c_{s-1}, c_s.  The CDF is
// nondecreasing along the chunk, so the entries <= tgt are a prefix and the
// first lane whose last entry exceeds tgt holds the crossing: one ballot per
// vector finds it and that lane's own count and bracket are read out -- no
// wave-wide reductions on the serial path.  Needs cb <= tgt < cb + the chunk's
// total (find_chunk guarantees it; zero-filled vectors past the row end then
// cannot be the first to exceed); returns false otherwise.
struct NoIdle {
    __device__ void operator()() {}
};
// `idle` runs once, right after the first round of loads is issued: work of the next
// step that the re-read's round trip can hide (k_decode_seq: its chunk-total scan).
template <typename E, int VEC, typename Idle = NoIdle>
__device__ inline bool scan_chunk(const E *row, int64_t nvec, int64_t cv0, int G, uint64_t cb, uint64_t tgt,
                                  uint64_t *cnt_out, uint64_t *lo_out, uint64_t *hi_out, Idle idle = Idle()) {
    constexpr int PF = 4;                                     // loads in flight: the scan is latency-bound
    for (int g0 = 0; g0 < G; g0 += PF) {
        typename VecT<E, VEC>::type xs[PF];
#pragma unroll
        for (int u = 0; u < PF; u++) {
            const int64_t vi = cv0 + (int64_t)(g0 + u) * 64 + (int64_t)lane_id();
            xs[u] = load_vec_or0<E, VEC>(row, g0 + u < G ? vi : nvec, nvec);
        }
        if (g0 == 0) idle();
#pragma unroll
        for (int u = 0; u < PF; u++) {
            if (g0 + u >= G) break;
            uint64_t loc[VEC], ls = 0;
#pragma unroll
            for (int j = 0; j < VEC; j++) { ls += (uint64_t)vget<E, VEC>(xs[u], j); loc[j] = ls; }
            const uint64_t in = wave_incl_scan_u64(ls);
            const uint64_t ex = cb + in - ls;                 // c just before this lane's entries
            const uint64_t mask = __ballot(ex + ls > tgt);
            if (mask) {
                const int L = __ffsll((unsigned long long)mask) - 1;
                uint64_t k = 0, lo = ex, hi = ~0ull;
#pragma unroll
                for (int j = 0; j < VEC; j++) {
                    const uint64_t ce = ex + loc[j];
                    const bool le = ce <= tgt;
                    k += le ? 1 : 0;
                    lo = le ? ce : lo;
                    hi = (!le && ce < hi) ? ce : hi;
                }
                *cnt_out = (uint64_t)((g0 + u) * 64 + L) * VEC + readlane_u64(k, L);
                *lo_out = readlane_u64(lo, L);
                *hi_out = readlane_u64(hi, L);
                return true;
            }
            cb += readlane_u64(in, 63);
        }
    }
    return false;
}

// Fudged val_to_symbol + symbol_to_range (fudged_dist closed form, lac_core.h
// fudge_f): f_e = e + g(Xmax_e), g(X) = max(1, min(C, floor(X / T))), C = w - V + 1,
// Xmax_e = max_{j<=e} (c_j w - j T), is strictly increasing, and val_to_symbol
// (bisect_right of floor(v*f_last/w) = v, arith_code.py:94-97) is the first e with
// f_e > v, i.e. with
//     e >= v   or   (v - e < C  and  Xmax_e >= (v - e + 1) T)
// -- one 128-bit product and compare per entry, no division.  One wave walks the
// row in chunks of 64 * VEC entries (one 16-B vector per lane, the next chunk in
// flight), the running maximum carried across chunks; the chunk holding s also
// holds Xmax_{s-1} and Xmax_s, so the range (f_{s-1}, f_s) needs no second pass
// and just two divisions.
template <typename E>
__device__ inline int decode_fudged(const E *row, int64_t V, uint64_t w, uint64_t v, uint64_t T, int64_t *s_out,
                                    uint64_t *a, uint64_t *bb) {
    constexpr int VEC = 16 / sizeof(E);
    const int lane = (int)lane_id();
    const int64_t C = (int64_t)(w - (uint64_t)V + 1);
    const int64_t nvec = (V + VEC - 1) / VEC;
    const bool vec_ok = (V % VEC) == 0 && ((uintptr_t)row & 15) == 0;
    auto load = [&](int64_t vi) {                           // entries past V read as 0
        typename VecT<E, 1>::type out[VEC];
        const int64_t e0 = vi * VEC;
        if (vec_ok && vi < nvec) {
            const typename VecT<E, VEC>::type x = load_vec<E, VEC>(row, vi);
#pragma unroll
            for (int j = 0; j < VEC; j++) out[j] = vget<E, VEC>(x, j);
        } else {
#pragma unroll
            for (int j = 0; j < VEC; j++) out[j] = e0 + j < V ? row[e0 + j] : (E)0;
        }
        struct R { E x[VEC]; } r;
#pragma unroll
        for (int j = 0; j < VEC; j++) r.x[j] = out[j];
        return r;
    };
    uint64_t base = 0;
    i128 xcarry = kI128Min;
    auto nxt = load(lane);
    for (int64_t r0 = 0; r0 < V; r0 += 64 * VEC) {
        const auto cur = nxt;
        if (r0 + 64 * VEC < V) nxt = load((r0 + 64 * VEC) / VEC + lane);
        uint64_t ls = 0;
#pragma unroll
        for (int j = 0; j < VEC; j++) ls += (uint64_t)cur.x[j];
        const uint64_t incl = wave_incl_scan_u64(ls);
        uint64_t c = base + incl - ls;
        i128 run[VEC], lm = kI128Min;
#pragma unroll
        for (int j = 0; j < VEC; j++) {
            const int64_t e = r0 + lane * VEC + j;
            c += (uint64_t)cur.x[j];
            const i128 X = e < V ? fudge_x(c, e, w, T) : kI128Min;
            lm = X > lm ? X : lm;
            run[j] = lm;                                      // lane-local prefix max
        }
        // exclusive wave max-scan of the lane maxima, after the carry
        const i128 pre = wave_incl_max_i128(lm);
        const i128 tot = readlane_i128(pre, 63);
        i128 excl = shfl_i128(pre, lane ? lane - 1 : 0);
        excl = lane ? (excl > xcarry ? excl : xcarry) : xcarry;
        int hit = -1;
#pragma unroll
        for (int j = VEC - 1; j >= 0; j--) {
            const int64_t e = r0 + lane * VEC + j;
            const i128 xm = run[j] > excl ? run[j] : excl;
            bool ok = e < V && (e >= (int64_t)v);
            if (e < V && !ok && (int64_t)v - e < C)
                ok = xm >= (i128)((u128)(uint64_t)((int64_t)v - e + 1) * T);
            hit = ok ? j : hit;
        }
        const uint64_t mask = __ballot(hit >= 0);
        if (mask) {
            const int L = __ffsll((unsigned long long)mask) - 1;
            const int jh = __shfl(hit, L);
            const int64_t s = r0 + (int64_t)L * VEC + jh;
            // Xmax_{s-1} and Xmax_s from lane L's registers
            i128 xprev = excl, xs = excl;
#pragma unroll
            for (int j = 0; j < VEC; j++) {
                const i128 xm = run[j] > excl ? run[j] : excl;
                if (j == jh - 1) xprev = xm;
                if (j == jh) xs = xm;
            }
            xprev = shfl_i128(xprev, L);
            xs = shfl_i128(xs, L);
            *a = s > 0 ? fudge_f(s - 1, xprev, T, w, V) : 0;
            *bb = fudge_f(s, xs, T, w, V);
            *s_out = s;
            return 0;
        }
        base += readlane_u64(incl, 63);
        xcarry = tot > xcarry ? tot : xcarry;
    }
    return LAC_E_DECODE_RANGE;
}

// Narrow to symbol s and renormalise, pulling k fresh bits into x
// (emit_symbol + emit_bit, arith_code.py:274-291, value form).  UNI: the state is
// wave-uniform (SGPRs) and the window words are read back from the vector loads that
// fetched them, so the renormalisation stays on the scalar unit.
template <bool UNI = false>
__device__ inline int decode_advance(DecState &st, uint64_t a, uint64_t bb, const BitWin &win, uint64_t nbits,
                                     int prec) {
    const int64_t l = st.l, x = st.x;
    if (!((l + (int64_t)a) <= x && x <= l + (int64_t)bb - 1)) return LAC_E_DECODE_RANGE;  // :277-278
    int64_t nl = l + (int64_t)a, nh = l + (int64_t)bb - 1;
    int k;
    uint64_t Ev;
    renorm(nl, nh, prec, &k, &Ev);
    int64_t nx = x;
    if (k > 0) {
        const int sh = prec - k;
        const BitWin wu = UNI ? BitWin{rfl_u64(win.w0), rfl_u64(win.w1)} : win;
        nx = (int64_t)((((uint64_t)x - (Ev << sh)) << k) | window_bits(wu, nbits, st.pos, k));
        st.pos += (uint64_t)k;
    }
    st.l = nl;
    st.h = nh;
    st.x = nx;
    st.nsym++;
    return 0;
}

#ifndef LAC_Q1D_NB
#define LAC_Q1D_NB 1             // k_q1_decode and k_decode_seq: decode_advance_nb (no renormalisation branches)
#endif
// decode_advance<true> with no branch past its range test (k_q1_decode, LAC_Q1D_NB):
// renorm()'s kk <= 0 case as kk = 0 (e = 0 keeps the registers), window_bits_nb.
__device__ inline int decode_advance_nb(DecState &st, uint64_t a, uint64_t bb, const BitWin &win, uint64_t nbits,
                                        int prec) {
    const int64_t l = st.l, x = st.x;
    if (!((l + (int64_t)a) <= x && x <= l + (int64_t)bb - 1)) return LAC_E_DECODE_RANGE;  // :277-278
    int64_t nl = l + (int64_t)a, nh = l + (int64_t)bb - 1;
    const uint64_t d = (uint64_t)(nh - nl);
    const int sh = bitlen64(d), k0 = prec - sh, k = k0 > 0 ? k0 : 0;
    const uint64_t Ev = k > 0 ? (uint64_t)nl >> sh : 0;
    nl = (int64_t)(((uint64_t)nl - (Ev << (sh & 63))) << k);
    nh = nl + (int64_t)((d + 1) << k) - 1;
    const BitWin wu{rfl_u64(win.w0), rfl_u64(win.w1)};
    st.x = (int64_t)((((uint64_t)x - (Ev << (sh & 63))) << k) | window_bits_nb(wu, nbits, st.pos, k));
    st.pos += (uint64_t)k;
    st.l = nl;
    st.h = nh;
    st.nsym++;
    return 0;
}

// Per-phase cycle accounting of the sequential decode step (tools/dec_phase_probe.sh
// builds a separate library with -DLAC_DEC_PHASES=1; the product build passes no clock
// and the marks compile to nothing).  Phases: 0 row totals + scan, 1 targets, 2 chunk
// search, 3 re-read + scan of the chunk, 4 ranges, 5 narrowing + renormalisation.
// (NoClock / PhaseClock: lac_dev.h)
#ifndef LAC_DEC_PHASES
#define LAC_DEC_PHASES 0
#endif
#if LAC_DEC_PHASES
__device__ unsigned long long g_dec_phase[8];
#endif

// r < 0 for a wave-uniform int64.  (Forcing the test onto the scalar unit -- the high
// word's sign through an opaque SGPR, or through readfirstlane -- measured slower in both
// sequential decoders, c2 1.29 -> 1.43 / 1.50 us/step, profiles/r04/lean/: the vector
// compare it replaces overlaps.)
__device__ inline bool neg_u(uint64_t r) { return (int64_t)r < 0; }

// div_small_fix for wave-uniform values (|r| < 3d < 2^53).
#ifndef LAC_DIVFIX_MASK
#define LAC_DIVFIX_MASK 1        // div_small_fix_u as sign masks (lac_core.h div_small_fix_mask), no loops
#endif
// MASK: the branch-free correction -- for the lone-wave chains (k_decode_lean, k_decode_seq:
// c2 decode 1.253 -> 1.229 us per step); k_q1_decode, whose 16 stream-waves per CU hide the
// loops' branches, keeps the loops (the masks' extra instructions: 4.3 -> 4.6 us per bf16 c3
// step; profiles/r05/straight/)
template <bool MASK = LAC_DIVFIX_MASK>
__device__ inline uint64_t div_small_fix_u(uint64_t q, uint64_t n, uint64_t m, uint64_t add, uint64_t d) {
    if constexpr (MASK) return div_small_fix_mask(q, n, m, add, d);
    uint64_t r = n * m + add - q * d;
    // (corrections as a fixed count of selects instead of these loops, which are never
    // entered past their first test: c2 1.29 -> 1.48 us/step, profiles/r04/lean/)
    while (neg_u(r)) { q -= 1; r += d; }
    for (;;) {
        const uint64_t t = r - d;
        if (neg_u(t)) break;
        q += 1;
        r = t;
    }
    return q;
}

// div_small with wave-uniform arguments: the double estimate on the vector unit (the
// SALU has no FP64), read back, the 64-bit remainder and its corrections on the SALU.
template <bool MASK = LAC_DIVFIX_MASK>
__device__ inline uint64_t div_small_u(uint64_t n, uint64_t m, uint64_t add, uint64_t d, double inv) {
    return div_small_fix_u<MASK>(rfl_u64(div_small_est(n, m, add, inv)), n, m, add, d);
}
// Two of them with one divisor (the ranges ceil(lo*w/T), ceil(hi*w/T)): both estimates
// first, so the two FP64 chains overlap, then both corrections.
template <bool MASK = LAC_DIVFIX_MASK>
__device__ inline void div_small_u2(uint64_t n0, uint64_t n1, uint64_t m, uint64_t add, uint64_t d, double inv,
                                    uint64_t *q0, uint64_t *q1) {
    const uint64_t e0 = rfl_u64(div_small_est(n0, m, add, inv)), e1 = rfl_u64(div_small_est(n1, m, add, inv));
    *q0 = div_small_fix_u<MASK>(e0, n0, m, add, d);
    *q1 = div_small_fix_u<MASK>(e1, n1, m, add, d);
}

// div_near (lac_core.h div_near_fix) with wave-uniform arguments: the lean step's u32 rows
__device__ inline uint64_t div_near_u(uint64_t n, uint64_t m, uint64_t add, uint64_t d, double inv) {
    return div_near_fix(rfl_u64(div_small_est(n, m, add, inv)), n, m, add, d);
}
template <bool N32 = true>
__device__ inline void div_near_u2(uint64_t n0, uint64_t n1, uint64_t m, uint64_t add, uint64_t d, double inv,
                                   uint64_t *q0, uint64_t *q1) {
    const uint64_t e0 = rfl_u64(div_small_est(n0, m, add, inv)), e1 = rfl_u64(div_small_est(n1, m, add, inv));
    *q0 = div_near_fix<N32>(e0, n0, m, add, d);
    *q1 = div_near_fix<N32>(e1, n1, m, add, d);
}

// 1/d for a d below 2^52, converted by the 2^52 magic (small_to_f64) instead of a general
// u64 -> f64 conversion (the lean step's 1/w, w <= 2^50): recip's one Newton step, and
// recip2_small's two -- 1/d to ~1 ulp, for estimates whose quotient reaches 2^50 and must
// stay within one (div_near on u64 rows)
__device__ inline double recip_small(uint64_t d) {
    const double dd = small_to_f64(d);
    const double r = __builtin_amdgcn_rcp(dd);
    return __builtin_fma(r, __builtin_fma(-dd, r, 1.0), r);
}
__device__ inline double recip2_small(uint64_t d) {
    const double dd = small_to_f64(d), r = recip_small(d);
    return __builtin_fma(r, __builtin_fma(-dd, r, 1.0), r);
}

// div_mid (lac_core.h) with wave-uniform arguments and div_mid_est_w's estimates (m < 2^52,
// the addend also as the double addd), both of a pair's estimates first so their FP64
// chains overlap: the lean step's ranges on u64 rows with totals >= 2^50.
__device__ inline void div_mid_u2(uint64_t n0, uint64_t n1, uint64_t m, uint64_t add, double addd, uint64_t d,
                                  double inv, uint64_t *q0, uint64_t *q1) {
    const uint64_t e0 = rfl_u64(div_mid_est_w(n0, m, addd, inv)), e1 = rfl_u64(div_mid_est_w(n1, m, addd, inv));
    *q0 = div_mid_fix(e0, n0, m, add, d);
    *q1 = div_mid_fix(e1, n1, m, add, d);
}

// Everything after the row's totals are known: val_to_symbol + symbol_to_range
// + advance.  `find_chunk(tgt, &cv0, &G, &cb)` locates the chunk holding tgt.
// UNI: the decoder state is wave-uniform (held in SGPRs by the caller), so the
// serial chain runs on the scalar unit with div_small's quotients where they are
// below 2^50 (prec <= 50, totals < 2^50): the few-stream decoders' step.
template <typename E, int VEC, typename FindChunk, bool UNI = false, typename Clock = NoClock, typename Idle = NoIdle>
__device__ inline int decode_symbol(DecState &st, const E *row, int64_t V, uint64_t T, uint64_t minp, int prec,
                                    int mapping, const uint8_t *bits, uint64_t nbits, FindChunk find_chunk,
                                    int64_t *s_out, Clock *clk = nullptr, Idle idle = Idle(),
                                    bool stop_undet = false) {
    auto mark = [&](int k) {
        if (clk) clk->mark(k);
    };
    const BitWin win = bit_window(bits, nbits, st.pos);       // in flight during the search
    const int64_t l = st.l, h = st.h, x = st.x;
    if (x < l || x > h) return LAC_E_DECODE_RANGE;            // corrupted state / bits
    const uint64_t w = (uint64_t)(h - l + 1), v = (uint64_t)(x - l);
    int64_t s = -1;
    uint64_t a = 0, bb = 0;
    // The reference decoder holds [lb, hb]: the bits read so far padded with 0s
    // and with 1s.  x is the 0-padded end; the 1-padded end adds 2^u - 1 where u
    // counts window bits past the end of the stream.  A symbol is "determined"
    // (decide_symbol's ls == hs, arith_code.py:268-273) iff both ends map to it.
    const uint64_t past = st.pos > nbits ? st.pos - nbits : 0;
    const int u = past < (uint64_t)prec ? (int)past : prec;
    const uint64_t vhi = v + ((1ull << u) - 1);
    bool det;
    if (mapping == LAC_MAP_FLOOR || !is_fudged(T, w, minp)) {
        uint64_t tgt, thi;                                    // targets of the 0- and 1-padded ends
        const bool small = UNI && T < kSmallQuot && prec <= 50;   // uniform
        if (small) {
            const double iw = recip(w);
            tgt = div_small_u(v, T, 0, w, iw);
            thi = vhi == v ? tgt : (vhi < w ? div_small_u(vhi, T, 0, w, iw) : 0);
        } else {
            div_pair(v, vhi < w ? vhi : 0, T, 0, w, recip(w), &tgt, &thi);   // tgt < T
        }
        mark(1);
        int64_t cv0;
        int G;
        uint64_t cb;
        if (!find_chunk(tgt, &cv0, &G, &cb)) return LAC_E_DECODE_RANGE;
        mark(2);
        uint64_t cnt, lo_c, hi_c;
        if (!scan_chunk<E, VEC>(row, V / VEC, cv0, G, cb, tgt, &cnt, &lo_c, &hi_c, idle)) return LAC_E_DECODE_RANGE;
        mark(3);
        s = cv0 * VEC + (int64_t)cnt;
        const uint64_t add = mapping == LAC_MAP_FLOOR ? 0 : T - 1;
        if (small) {
            div_small_u2(lo_c, hi_c, w, add, T, recip(T), &a, &bb);
        } else {
            div_pair(lo_c, hi_c, w, add, T, recip(T), &a, &bb);
        }
        mark(4);
        det = vhi < w && thi < hi_c;                          // bisect_right(cdf, t_hi) == s
    } else {
        const int e = decode_fudged<E>(row, V, w, v, T, &s, &a, &bb);
        if (e) return e;
        if (UNI) {                  // (from the wave reductions: back to SGPRs)
            a = rfl_u64(a);
            bb = rfl_u64(bb);
            s = (int64_t)rfl_u64((uint64_t)s);
        }
        det = vhi < bb;                                       // f_s > v_hi
    }
    // LAC_OPT_DECODE_STOP: the stream stops before the first symbol its bits do not
    // determine, registers unchanged (the drop-in decoder parks there, lac_amd.coder)
    if (stop_undet && !det) return LAC_E_UNDETERMINED;
    if (st.det && det) st.ndet++;
    else st.det = 0;
    *s_out = s;
    // (UNI, the lone-wave k_decode_seq: the renormalisation without branches, as k_q1_decode)
    const int rc = (UNI && LAC_Q1D_NB) ? decode_advance_nb(st, a, bb, win, nbits, prec)
                                        : decode_advance<UNI>(st, a, bb, win, nbits, prec);
    mark(5);
    return rc;
}


}  // namespace
