// lac_decode.hip -- the decode family of liblac.so: A_from_bin (arith_code.py:248-334)
// in value-register form.  Per step the row is streamed into totals, the search finds
// the chunk holding floor((x-l)*T/w), only that chunk is re-read and scanned to the
// symbol (val_to_symbol's bisect_right, :94-97), and the value window advances by the
// renormalisation (emit_bit, :284-291).  At >= 2048 streams one launch per job with
// one wave per stream (k_decode_wave_fine); fewer streams take the block and stats
// paths (k_decode_block; k_dec_stats + k_decode_seq / k_decode_lean); the flush and
// windows that leave [l, h] run in the reference's own frame (lac_tail.h).
#include <type_traits>

#include "lac_host.h"
#include "lac_dec_dev.h"

namespace {

// One decode step for every stream, NW waves per stream (small stream counts:
// with few streams the row of one stream must be streamed by many waves).
template <typename E, int VEC, int G, int NW>
__global__ __launch_bounds__(64 * NW) void k_decode_step(const E *__restrict__ pmf, int64_t step_off,
                                                         int64_t stream_stride, int64_t V, int prec,
                                                         DecState *states, const uint8_t *bits, uint64_t stride,
                                                         const uint64_t *nbits, int32_t *sym_out, int64_t B,
                                                         int mapping) {
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    __shared__ uint64_t wmin[NW];
    __shared__ uint32_t wovf[NW];
    const int lane = (int)lane_id(), wave = threadIdx.x >> 6;
    const int64_t b = blockIdx.x;
    DecState st = states[b];
    if (st.err) {
        if (threadIdx.x == 0) sym_out[b] = -1;
        return;
    }
    const E *row = pmf + step_off + b * stream_stride;
    constexpr int64_t CH = 64 * VEC * G;                 // elements per chunk
    const int64_t nvec = V / VEC, nch = (V + CH - 1) / CH;
    uint64_t *csum = smem;
    // ---- pass 1: chunk sums, minp (all waves)
    uint64_t mn = ~0ull;
    uint32_t ovf = 0;
    for (int64_t c = wave; c < nch; c += NW) {
        uint64_t ls = 0;
        typename VecT<E, VEC>::type x[G];
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int64_t vi = c * 64 * G + g * 64 + lane;
            x[g] = load_vec_or0<E, VEC>(row, vi, nvec);
        }
#pragma unroll
        for (int g = 0; g < G; g++) {
#pragma unroll
            for (int j = 0; j < VEC; j++) {
                const uint64_t e = (uint64_t)vget<E, VEC>(x[g], j);
                const uint64_t n2 = ls + e;
                ovf |= n2 < ls;
                ls = n2;
                const uint64_t m1 = e - 1;
                mn = m1 < mn ? m1 : mn;
            }
        }
        uint64_t tsum = ls;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            const uint64_t o = shfl_xor_u64(tsum, m);
            const uint64_t n2 = tsum + o;
            ovf |= n2 < tsum;
            tsum = n2;
        }
        if (lane == 0) csum[c] = tsum;
    }
    mn = wave_min_u64(mn);
    ovf = (uint32_t)__any(ovf);
    if (lane == 0) { wmin[wave] = mn; wovf[wave] = ovf; }
    __syncthreads();
    if (wave != 0) return;
    // ---- wave 0: T, minp, chunk prefix
    uint64_t m0 = wmin[0];
    uint32_t anyovf = wovf[0];
    for (int i = 1; i < NW; i++) { m0 = wmin[i] < m0 ? wmin[i] : m0; anyovf |= wovf[i]; }
    const int64_t per = (nch + 63) / 64;
    const int64_t c0 = lane * per, c1 = (c0 + per < nch) ? c0 + per : nch;
    u128 local = 0;
    for (int64_t c = c0; c < c1; c++) local += csum[c];
    const u128 tot = wave_sum_u128(local);
    const uint64_t incl = wave_incl_scan_u64((uint64_t)local);
    int err = 0;
    if (__any(anyovf) || (tot >> 64) || tot == 0) err = LAC_E_TABLE;
    int64_t s = -1;
    if (!err) {
        auto find_chunk = [&](uint64_t tgt, int64_t *cv0, int *g, uint64_t *cb) {
            uint64_t run = incl - (uint64_t)local;
            int64_t fc = -1;
            uint64_t fbase = 0;
            for (int64_t c = c0; c < c1; c++) {
                const uint64_t nx = run + csum[c];
                if (fc < 0 && run <= tgt && tgt < nx) { fc = c; fbase = run; }
                run = nx;
            }
            const uint64_t mask = __ballot(fc >= 0);
            if (!mask) return false;
            const int src = __ffsll((unsigned long long)mask) - 1;
            *cv0 = (int64_t)readlane_u64((uint64_t)fc, src) * 64 * G;
            *g = G;
            *cb = readlane_u64(fbase, src);
            return true;
        };
        err = decode_symbol<E, VEC>(st, row, V, (uint64_t)tot, m0 + 1, prec, mapping, bits + b * stride, nbits[b],
                                    find_chunk, &s);
    }
    if (lane == 0) {
        if (err) {
            st.err = err;
            st.err_step = st.nsym;
        }
        sym_out[b] = err ? -1 : (int32_t)s;
        states[b] = st;
    }
}

// Decode `nsteps` steps of every stream in one launch, one wave per stream
// (large stream counts).  Pass 1 streams the row (8 x 16-B loads in flight
// per lane) into <= 64 chunk totals, chunk c's total kept by lane c; the
// search is a wave scan over lanes; only the chunk holding the target is
// re-read.  Serial per-stream work is hidden behind the other waves' loads.
template <typename E, int VEC>
__global__ LAC_DEC_BOUNDS void k_decode_wave(const E *__restrict__ pmf, int64_t step_stride,
                                                     int64_t stream_stride, int64_t nsteps, int64_t V, int prec,
                                                     DecState *states, const uint8_t *bits, uint64_t stride,
                                                     const uint64_t *nbits, int32_t *sym_out, int64_t B,
                                                     int mapping) {
    const int lane = (int)lane_id();
    const int64_t b = (int64_t)blockIdx.x * kStreamWaves + wave_in_block();
    if (b >= B) return;
    DecState st = states[b];
    const uint8_t *mybits = bits + b * stride;
    const uint64_t mynbits = nbits[b];
    const int64_t nvec = V / VEC, nit = (nvec + 63) / 64;
    constexpr int U = 8;
    int64_t CI = (nit + 63) / 64;                             // iterations per chunk: <= 64 chunks
    CI = ((CI + U - 1) / U) * U;
    const int64_t nch = (nit + CI - 1) / CI;
    for (int64_t t = 0; t < nsteps; t++) {
        int32_t *out = sym_out + t * B + b;
        if (st.err) {
            if (lane == 0) *out = -1;
            continue;
        }
        const E *row = pmf + t * step_stride + b * stream_stride;
        uint64_t mine = 0;
        E mn = (E)~(E)0;
        uint32_t ovf = 0;
        for (int64_t c = 0; c < nch; c++) {
            uint64_t acc = 0;
            for (int64_t g0 = 0; g0 < CI; g0 += U) {
                typename VecT<E, VEC>::type x[U];
                const bool full = (c * CI + g0 + U) * 64 <= nvec;
                if (full) {
#pragma unroll
                    for (int u = 0; u < U; u++) x[u] = load_vec<E, VEC>(row, (c * CI + g0 + u) * 64 + lane);
                } else {
#pragma unroll
                    for (int u = 0; u < U; u++) x[u] = load_vec_or0<E, VEC>(row, (c * CI + g0 + u) * 64 + lane, nvec);
                }
#pragma unroll
                for (int u = 0; u < U; u++) {
#pragma unroll
                    for (int j = 0; j < VEC; j++) {
                        const E e = vget<E, VEC>(x[u], j);
                        if constexpr (sizeof(E) == 8) {       // u64 rows can overflow; u32 chunks cannot
                            const uint64_t n2 = acc + e;
                            ovf |= n2 < acc;
                            acc = n2;
                        } else {
                            acc += e;
                        }
                        const E m1 = e - 1;
                        mn = m1 < (E)mn ? m1 : (E)mn;
                    }
                }
            }
            uint64_t tsum = acc;
            if constexpr (sizeof(E) == 8) {
#pragma unroll
                for (int m = 32; m >= 1; m >>= 1) {
                    const uint64_t o = shfl_xor_u64(tsum, m);
                    const uint64_t n2 = tsum + o;
                    ovf |= n2 < tsum;
                    tsum = n2;
                }
            } else {
                tsum = wave_sum_u64(tsum);                    // < 2^32 * 2^31: no overflow
            }
            if (lane == c) mine = tsum;
        }
        uint64_t minp;
        if constexpr (sizeof(E) == 8) minp = wave_min_u64(mn) + 1;
        else minp = (uint64_t)wave_min_u32(mn) + 1;
        const uint64_t incl = wave_incl_scan_u64(mine);
        const u128 acc128 = wave_sum_u128((u128)mine);
        int err = 0;
        if (__any(ovf) || (acc128 >> 64) || acc128 == 0) err = LAC_E_TABLE;
        int64_t s = -1;
        if (!err) {
            auto find_chunk = [&](uint64_t tgt, int64_t *cv0, int *g, uint64_t *cb) {
                const uint64_t ex = incl - mine;
                const bool hit = lane < nch && ex <= tgt && tgt < incl;
                const uint64_t mask = __ballot(hit);
                if (!mask) return false;
                const int src = __ffsll((unsigned long long)mask) - 1;
                *cv0 = (int64_t)src * CI * 64;
                *g = (int)CI;
                *cb = readlane_u64(ex, src);
                return true;
            };
            err = decode_symbol<E, VEC>(st, row, V, (uint64_t)acc128, minp, prec, mapping, mybits, mynbits,
                                        find_chunk, &s);
        }
        if (err) {
            st.err = err;
            st.err_step = st.nsym;
        }
        if (lane == 0) *out = err ? -1 : (int32_t)s;
    }
    if (lane == 0) states[b] = st;
}

// 64-bit partner exchange across lane bit BIT (DPP inside a 16-lane row, a
// ds_bpermute swizzle across rows).
template <int BIT>
__device__ inline uint64_t xor_lane_u64(uint64_t x) {
    if constexpr (BIT < 4) return ((uint64_t)xor_dpp<BIT>((uint32_t)(x >> 32)) << 32) | xor_dpp<BIT>((uint32_t)x);
    else return shfl_xor_u64(x, 1 << BIT);
}
// ---- row totals and minp without 64-bit compares on the streaming loop
// u64 rows: the total is accumulated wrapping mod 2^64 next to H = the sum of the
// entries' high words (exact).  T lies in [2^32 H, 2^32 (H + V)) and V <= 2^31,
// so T = S + k 2^64 with k in {0, 1} (S the wrapped sum), and T < 2^64 iff
// H < 2^32 and S >= 2^32 H.  While T < 2^64 every partial sum is exact.
__device__ inline bool u64_total_overflows(uint64_t S, uint64_t H) { return (H >> 32) || S < (H << 32); }

// minp key: e - 1 (0 wraps to the max, as CDFPredictor.minp skips zeros,
// arith_code.py:79-82); for u64 entries >= 2^32 the key saturates, so one 32-bit
// min per entry finds every minp below 2^32 exactly.
template <typename E> __device__ inline uint32_t min_key(E e);
template <> __device__ inline uint32_t min_key<uint32_t>(uint32_t e) { return e - 1u; }
template <> __device__ inline uint32_t min_key<uint64_t>(uint64_t e) {
    return (e >> 32) ? 0xFFFFFFFFu : (uint32_t)e - 1u;
}

// minp from the row's minimum key (wave-uniform).  Exact, except that a u64 row
// whose positive entries are all >= 2^32 reports 2^32: minp only enters the
// fudge test T > w * minp (arith_code.py:84), which 2^32 decides exactly unless
// T > w * 2^32 (possible below prec 34 only) -- then the row is re-scanned with
// 64-bit mins (cold).
template <typename E>
__device__ inline uint64_t row_minp(const E *row, int64_t V, uint32_t kmin, uint64_t T, uint64_t w) {
    if constexpr (sizeof(E) == 8) {
        if (kmin == 0xFFFFFFFFu && (u128)T > ((u128)w << 32)) {
            uint64_t m = ~0ull;
            for (int64_t i = lane_id(); i < V; i += 64) { const uint64_t e = row[i] - 1; m = e < m ? e : m; }
            return wave_min_u64(m) + 1;
        }
    }
    (void)row; (void)V; (void)T; (void)w;
    return (uint64_t)kmin + 1;
}

template <bool CHK>
__device__ inline uint64_t add_ovf(uint64_t a, uint64_t b, uint32_t &ovf) {
    const uint64_t s = a + b;
    if constexpr (CHK) ovf |= s < a;
    return s;
}

// Totals of 8 per-lane values s[0..7] over the wave, all 8 at once: halving
// exchanges over lane bits 0..2 (DPP), then full sums over bits 3..5.  Lane l
// ends with the total of s[l & 7] (the inputs are fed bit-reversed, so the
// halving's reversed index order comes out straight).  CHK tracks u64 wrap.
template <bool CHK>
__device__ inline uint64_t wave_sum8_u64(const uint64_t (&s)[8], uint32_t &ovf) {
    const int lane = (int)lane_id();
    uint64_t v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = s[((i & 1) << 2) | (i & 2) | ((i >> 2) & 1)];
    {
        const bool up = lane & 1;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint64_t keep = up ? v[i + 4] : v[i], give = up ? v[i] : v[i + 4];
            v[i] = add_ovf<CHK>(keep, xor_lane_u64<0>(give), ovf);
        }
    }
    {
        const bool up = lane & 2;
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const uint64_t keep = up ? v[i + 2] : v[i], give = up ? v[i] : v[i + 2];
            v[i] = add_ovf<CHK>(keep, xor_lane_u64<1>(give), ovf);
        }
    }
    {
        const bool up = lane & 4;
        const uint64_t keep = up ? v[1] : v[0], give = up ? v[0] : v[1];
        v[0] = add_ovf<CHK>(keep, xor_lane_u64<2>(give), ovf);
    }
    uint64_t r = v[0];
    r = add_ovf<CHK>(r, xor_lane_u64<3>(r), ovf);
    r = add_ovf<CHK>(r, xor_lane_u64<4>(r), ovf);
    r = add_ovf<CHK>(r, xor_lane_u64<5>(r), ovf);
    return r;
}

#ifndef LAC_DEC_XPF                // k_decode_wave_fine: next group in flight while one is consumed,
                                   // and the next row's first group over the step's tail (+2.5 %)
#define LAC_DEC_XPF 1
#endif
#ifndef LAC_DEC_STREAM_ONLY        // timing experiment only: skip the search (wrong symbols)
#define LAC_DEC_STREAM_ONLY 0
#endif

// k_decode_wave with one total per 64-vector iteration of the row instead of per
// <= 64-iteration chunk (rows of <= 512 iterations: V <= 131072 u32 / 65536 u64
// entries).  Iteration p's total lives in lane p % 64 of register p / 64, the
// search scans those NR registers, and the re-read after the search is ONE 16-B
// load per lane (1 KB, 0.8 % of a 32000-entry u32 row) instead of a chunk of
// eight (6.3 %), which also shortens the dependent tail of every step.
template <typename E, int VEC, int NR>
__global__ __launch_bounds__(64 * LAC_STREAM_WG, LAC_DECF_MINW) void k_decode_wave_fine(const E *__restrict__ pmf, int64_t step_stride,
                                                  int64_t stream_stride, int64_t nsteps, int64_t V, int prec,
                                                  DecState *states, const uint8_t *bits, uint64_t stride,
                                                  const uint64_t *nbits, int32_t *sym_out, int64_t B, int mapping) {
    constexpr bool W = sizeof(E) == 8;
    const int lane = (int)lane_id();
    const int64_t b = (int64_t)blockIdx.x * kStreamWaves + wave_in_block();
    if (b >= B) return;
    DecState st = states[b];
    const uint8_t *mybits = bits + b * stride;
    const uint64_t mynbits = nbits[b];
    const int nvec = (int)(V / VEC), nit = (nvec + 63) / 64, ngrp = (nit + 7) / 8;
#if LAC_DEC_XPF
    // XD = 2: two groups in flight (g + 1 and g + 2) while group g is summed, and the
    // next row's groups 0 and 1 over the step's tail; rows of <= 128 iterations (u64:
    // <= 256) only (240-250 VGPRs; longer u32 rows' second buffer spilled)
    constexpr int XD = (LAC_DEC_XPF >= 2 && (NR <= 2 || (W && NR <= 4))) ? 2 : 1;
    typename VecT<E, VEC>::type xb[8], xb2[8];
    if (nsteps > 0) {
        const E *row0 = pmf + b * stream_stride;
#pragma unroll
        for (int u = 0; u < 8; u++)
            xb[u] = nvec >= 512 ? load_vec<E, VEC>(row0, u * 64 + lane) : load_vec_or0<E, VEC>(row0, u * 64 + lane, nvec);
        if (XD == 2 && ngrp > 1) {
#pragma unroll
            for (int u = 0; u < 8; u++)
                xb2[u] = nvec >= 1024 ? load_vec<E, VEC>(row0, (8 + u) * 64 + lane)
                                      : load_vec_or0<E, VEC>(row0, (8 + u) * 64 + lane, nvec);
        }
    }
#endif
    for (int64_t t = 0; t < nsteps; t++) {
        int32_t *out = sym_out + t * B + b;
        if (st.err) {
            if (lane == 0) *out = -1;
            continue;
        }
        const E *row = pmf + t * step_stride + b * stream_stride;
        uint64_t mine[NR];
#pragma unroll
        for (int r = 0; r < NR; r++) mine[r] = 0;
        uint32_t mn = ~0u;                                    // min over min_key (0 -> max)
        uint32_t hh = 0;                                      // u64 rows: sum of the high words, saturating
                                                              // (a lane at 2^32 - 1 already means T >= 2^64)
        uint32_t ovf = 0;                                     // (unused: totals wrap, see u64_total_overflows)
        const int nfull = nvec / 512;                         // groups of 8 whole iterations
        auto group = [&](int g, bool full) {
#if LAC_DEC_XPF
            // x holds group g (issued after group g-1, or before the previous step's tail)
            typename VecT<E, VEC>::type x[8];
#pragma unroll
            for (int u = 0; u < 8; u++) x[u] = xb[u];
            if constexpr (XD == 2) {
#pragma unroll
                for (int u = 0; u < 8; u++) xb[u] = xb2[u];
            }
            auto &nb = XD == 2 ? xb2 : xb;                    // group g + XD into the freed buffer
            if (g + XD < ngrp) {
                const bool nf = g + XD < nfull;
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int vi = ((g + XD) * 8 + u) * 64 + lane;
                    nb[u] = nf ? load_vec<E, VEC>(row, vi) : load_vec_or0<E, VEC>(row, vi, nvec);
                }
            }
#else
            typename VecT<E, VEC>::type x[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int vi = (g * 8 + u) * 64 + lane;
                x[u] = full ? load_vec<E, VEC>(row, vi) : load_vec_or0<E, VEC>(row, vi, nvec);
            }
#endif
            uint64_t s[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                uint64_t a = 0;
#pragma unroll
                for (int j = 0; j < VEC; j++) {
                    const E e = vget<E, VEC>(x[u], j);
                    a += (uint64_t)e;                         // wraps only if T >= 2^64 (detected below)
                    // one clamped v_add_u32 (a 64-bit sum took a move and a 64-bit add)
                    if constexpr (W) hh = __builtin_elementwise_add_sat(hh, (uint32_t)((uint64_t)e >> 32));
                }
                if constexpr (W) {                            // VEC = 2: both keys in one v_min3_u32
                    mn = min(mn, min(min_key<E>(vget<E, VEC>(x[u], 0)), min_key<E>(vget<E, VEC>(x[u], 1))));
                } else {
#pragma unroll
                    for (int j = 0; j < VEC; j++) mn = min(mn, min_key<E>(vget<E, VEC>(x[u], j)));
                }
                s[u] = a;
            }
            const uint64_t tot = wave_sum8_u64<false>(s, ovf);   // lane l: iteration g*8 + (l & 7)
            const bool mylane = (lane >> 3) == (g & 7);
#pragma unroll
            for (int r = 0; r < NR; r++)
                if (r == (g >> 3) && mylane) mine[r] = tot;
        };
        for (int g = 0; g < nfull; g++) group(g, true);
        if (nfull < ngrp) group(nfull, false);
#if LAC_DEC_XPF
        if (t + 1 < nsteps) {                                 // next row's group 0, in flight over the tail
            const E *nrow = row + step_stride;
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int vi = u * 64 + lane;
                xb[u] = nfull > 0 ? load_vec<E, VEC>(nrow, vi) : load_vec_or0<E, VEC>(nrow, vi, nvec);
            }
            if (XD == 2 && ngrp > 1) {                        // and its group 1
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int vi = (8 + u) * 64 + lane;
                    xb2[u] = nfull > 1 ? load_vec<E, VEC>(nrow, vi) : load_vec_or0<E, VEC>(nrow, vi, nvec);
                }
            }
        }
#endif
        uint64_t incl[NR];
        uint64_t base = 0;
#pragma unroll
        for (int r = 0; r < NR; r++) {
            incl[r] = base + wave_incl_scan_u64(mine[r]);     // exact once T < 2^64 is checked
            base = readlane_u64(incl[r], 63);
        }
        const uint64_t T = base;
        int err = 0;
        if (T == 0) err = LAC_E_TABLE;
        if constexpr (W) { if (u64_total_overflows(T, wave_sum_u64((uint64_t)hh))) err = LAC_E_TABLE; }
        const uint64_t minp = err ? 1 : row_minp<E>(row, V, wave_min_u32(mn), T, (uint64_t)(st.h - st.l + 1));
        int64_t s = -1;
        if (!err) {
            auto find_chunk = [&](uint64_t tgt, int64_t *cv0, int *G, uint64_t *cb) {
#pragma unroll
                for (int r = 0; r < NR; r++) {
                    const uint64_t ex = incl[r] - mine[r];
                    const bool hit = r * 64 + lane < nit && ex <= tgt && tgt < incl[r];
                    const uint64_t mask = __ballot(hit);
                    if (mask) {
                        const int src = __ffsll((unsigned long long)mask) - 1;
                        *cv0 = (int64_t)(r * 64 + src) * 64;
                        *G = 1;
                        *cb = readlane_u64(ex, src);
                        return true;
                    }
                }
                return false;
            };
            if (LAC_DEC_STREAM_ONLY) s = (int64_t)(minp & 1);
            else err = decode_symbol<E, VEC>(st, row, V, T, minp, prec, mapping, mybits, mynbits, find_chunk, &s);
        }
        if (err) {
            st.err = err;
            st.err_step = st.nsym;
        }
        if (lane == 0) *out = err ? -1 : (int32_t)s;
    }
    if (lane == 0) states[b] = st;
}

// ---------------------------------------------------------- decode, block path
// Fewer streams than fill the chip with one wave each: one NW-wave workgroup
// per stream, pipelined.  Waves 1..NW-1 ("streamers") stream row t+1 into
// per-iteration totals in LDS (groups of 8 iterations, k_decode_wave_fine's
// butterfly) while wave 0 (the coder) finishes step t from row t's totals:
// search, the one 16-B-per-lane re-read, renormalisation.  The rows do not
// depend on the decoder state, so only the totals cross between waves, double
// buffered, with one workgroup barrier per step.  NW = 4/8/16 keeps ~16 waves
// per CU from 1024 down to 256 streams.
template <typename E, int VEC, int NW>
__global__ __launch_bounds__(64 * NW) void k_decode_block(const E *__restrict__ pmf, int64_t step_stride,
                                                          int64_t stream_stride, int64_t nsteps, int64_t V, int prec,
                                                          DecState *states, const uint8_t *bits, uint64_t stride,
                                                          const uint64_t *nbits, int32_t *sym_out, int64_t B,
                                                          int mapping) {
    constexpr bool W = sizeof(E) == 8;
    constexpr int S = NW - 1, NRMAX = 8;                      // streamer waves; <= 512 iterations per row
    __shared__ uint64_t tot[2][64 * NRMAX];
    __shared__ uint64_t smin[2][S];
    __shared__ uint32_t sovf[2][S];
    __shared__ int32_t serr;
    const int lane = (int)lane_id(), w = wave_in_block();
    const int64_t b = blockIdx.x;
    const int nvec = (int)(V / VEC), nit = (nvec + 63) / 64, ngrp = (nit + 7) / 8;
    if (threadIdx.x == 0) serr = states[b].err;

    // streamer s (1..S): groups s-1, s-1+S, ... of step t into buffer t & 1
    auto stream_row = [&](int64_t t) {
        const E *row = pmf + t * step_stride + b * stream_stride;
        const int buf = (int)(t & 1);
        E mn = (E)~(E)0;
        uint32_t ovf = 0;
        for (int g = w - 1; g < ngrp; g += S) {
            typename VecT<E, VEC>::type x[8];
            const bool full = (g + 1) * 512 <= nvec;
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int vi = (g * 8 + u) * 64 + lane;
                x[u] = full ? load_vec<E, VEC>(row, vi) : load_vec_or0<E, VEC>(row, vi, nvec);
            }
            uint64_t s8[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                uint64_t a = 0;
#pragma unroll
                for (int j = 0; j < VEC; j++) {
                    const E e = vget<E, VEC>(x[u], j);
                    a = add_ovf<W>(a, (uint64_t)e, ovf);
                    const E m1 = e - 1;
                    mn = m1 < mn ? m1 : mn;
                }
                s8[u] = a;
            }
            const uint64_t gt = wave_sum8_u64<W>(s8, ovf);     // lane l: iteration g*8 + (l & 7)
            if (lane < 8 && g * 8 + lane < nit) tot[buf][g * 8 + lane] = gt;
        }
        uint64_t m64;
        if constexpr (W) m64 = wave_min_u64(mn);
        else m64 = wave_min_u32(mn);
        const uint32_t o = (uint32_t)__any(ovf);
        if (lane == 0) { smin[buf][w - 1] = m64; sovf[buf][w - 1] = o; }
    };

    DecState st;
    const uint8_t *mybits = bits + b * stride;
    uint64_t mynbits = 0;
    if (w == 0) { st = states[b]; mynbits = nbits[b]; }
    __syncthreads();
    const bool dead = serr != 0;                              // an errored stream stays errored
    if (w > 0 && !dead && nsteps > 0) stream_row(0);
    __syncthreads();
    for (int64_t t = 0; t < nsteps; t++) {
        if (w > 0) {
            if (!dead && t + 1 < nsteps) stream_row(t + 1);
        } else {
            int32_t *out = sym_out + t * B + b;
            if (st.err) {
                if (lane == 0) *out = -1;
            } else {
                const int buf = (int)(t & 1);
                const E *row = pmf + t * step_stride + b * stream_stride;
                uint64_t mine[NRMAX], incl[NRMAX];
                u128 lsum = 0;
                uint64_t base = 0, mn = ~0ull;
                uint32_t ovf = 0;
#pragma unroll
                for (int i = 0; i < S; i++) {
                    mn = smin[buf][i] < mn ? smin[buf][i] : mn;
                    ovf |= sovf[buf][i];
                }
#pragma unroll
                for (int r = 0; r < NRMAX; r++) {
                    const int p = r * 64 + lane;
                    mine[r] = (r * 64 < nit && p < nit) ? tot[buf][p] : 0;
                    lsum += mine[r];
                    incl[r] = base + wave_incl_scan_u64(mine[r]);
                    base = readlane_u64(incl[r], 63);
                }
                const u128 acc128 = W ? wave_sum_u128(lsum) : (u128)base;
                int err = 0;
                if (ovf || (acc128 >> 64) || acc128 == 0) err = LAC_E_TABLE;
                int64_t s = -1;
                if (!err) {
                    auto find_chunk = [&](uint64_t tgt, int64_t *cv0, int *G, uint64_t *cb) {
#pragma unroll
                        for (int r = 0; r < NRMAX; r++) {
                            const uint64_t ex = incl[r] - mine[r];
                            const bool hit = r * 64 + lane < nit && ex <= tgt && tgt < incl[r];
                            const uint64_t mask = __ballot(hit);
                            if (mask) {
                                const int src = __ffsll((unsigned long long)mask) - 1;
                                *cv0 = (int64_t)(r * 64 + src) * 64;
                                *G = 1;
                                *cb = readlane_u64(ex, src);
                                return true;
                            }
                        }
                        return false;
                    };
                    err = decode_symbol<E, VEC>(st, row, V, (uint64_t)acc128, mn + 1, prec, mapping, mybits, mynbits,
                                                find_chunk, &s);
                }
                if (err) {
                    st.err = err;
                    st.err_step = st.nsym;
                }
                if (lane == 0) *out = err ? -1 : (int32_t)s;
            }
        }
        __syncthreads();
    }
    if (w == 0 && lane == 0) states[b] = st;
}

// ---------------------------------------------------------- decode, stats path
// Few streams: the per-step kernels above leave the chip idle (one stream's row
// per step) and pay a launch per step.  The row statistics a decode step needs
// -- the <= 64 chunk totals of k_decode_wave's layout, T and minp -- do not
// depend on the decoder state, so k_dec_stats computes them for every (step,
// stream) row of a chunk of steps at once (one wave per row, the whole chip),
// and k_decode_seq walks each stream's steps touching only those 528 bytes plus
// the one chunk holding the target (1/64 of the row; fudged rows take
// decode_symbol's full-row form).
// load_vec_or0 with the default (cache-allocating) policy instead of nontemporal.
template <typename E, int VEC>
__device__ inline typename VecT<E, VEC>::type load_vec_keep(const E *row, int64_t vi, int64_t nvec) {
    typedef typename VecT<E, VEC>::type Vt;
    const bool ok = vi < nvec;
    const Vt x = reinterpret_cast<const Vt *>(row)[ok ? vi : nvec - 1];
    return ok ? x : (Vt)0;
}

struct DecRowMeta {
    uint64_t T;            // 0 marks a bad row (empty or total >= 2^64)
    uint64_t minp;
};

// Chunks of CI = ceil(iterations / 64) 64-vector iterations, the finest that
// keeps <= 64 totals (V = 32000 u32: 63 chunks of 2 iterations, so the per-step
// re-read is 2 vectors per lane, one round of loads).
template <typename E, int VEC>
__device__ inline void dec_chunk_layout(int64_t V, int64_t *CI, int64_t *nch) {
    const int64_t nvec = V / VEC, nit = (nvec + 63) / 64;
    const int64_t ci = nit ? (nit + 63) / 64 : 1;
    *CI = ci;
    *nch = (nit + ci - 1) / ci;
}

// The lean step's chunks: up to 64 * LeanCW<E> of them, LeanCW bounds per lane -- u64 rows
// two (V = 32000: 125 chunks of 2 iterations, two 16-B loads per lane and step instead of
// four), u32 rows one (the layout above).
#ifndef LAC_LEAN_CW32
#define LAC_LEAN_CW32 1          // (2 for u32 rows too: c2 0.849-0.851 vs 0.848-0.850 us, profiles/r06/lean3/cw32/)
#endif
template <typename E> constexpr int LeanCW = sizeof(E) == 8 ? 2 : LAC_LEAN_CW32;
typedef VecT<uint64_t, 2>::type u64x2;
template <typename E, int VEC>
__host__ __device__ inline void lean_chunk_layout(int64_t V, int64_t *CI, int64_t *nch) {
    const int64_t nvec = V / VEC, nit = (nvec + 63) / 64, per = 64 * LeanCW<E>;
    const int64_t ci = nit ? (nit + per - 1) / per : 1;
    *CI = ci;
    *nch = (nit + ci - 1) / ci;
}

// What k_decode_lean reads of a row (LEAN builds of k_dec_stats), besides its CDF:
struct LeanMeta {
    uint64_t T;            // the total; 0: not for the lean step (bad row, u32 total >= 2^32, minp 0)
    uint64_t fthr;         // ceil(T / minp): the ceil mapping's range is fudged iff w < fthr (arith_code.py:84)
    double iT;             // 1/T correctly rounded
    double Td;             // T rounded to a double (the wide rows' target window)
};
// Totals the lean step takes: below 2^32 for u32 tables (their CDF then fits the entries'
// own width); any valid total (below 2^64) for u64 tables, whose steps divide with
// div_small below 2^50 and with the 128-bit remainders of div_mid / div_floor_inv above.
template <typename E> __device__ inline bool lean_total_ok(uint64_t T) {
    return sizeof(E) == 8 || T < (1ull << 32);
}

// LEAN: also the row's per-entry CDF for k_decode_lean -- lcdf[row][i], the inclusive sum of
// the row's entries up to i in the entries' own width (mod 2^32 / 2^64) -- its chunks'
// exclusive bounds lchunk[row][lane] and a LeanMeta; exact where lean_total_ok.  (Round 6; rounds 4-5 wrote one CDF word per 16-B vector, and the step
// then loaded the pmf vector and that word and summed the vector itself.)
template <typename E, int VEC, bool LEAN = false>
__global__ __launch_bounds__(256) void k_dec_stats(const E *__restrict__ pmf, int64_t step_stride,
                                                   int64_t stream_stride, int64_t B, int64_t rows, int64_t V,
                                                   int64_t t0, uint64_t *__restrict__ chunks,
                                                   DecRowMeta *__restrict__ meta, E *__restrict__ lcdf = nullptr,
                                                   uint64_t *__restrict__ lchunk = nullptr,
                                                   LeanMeta *__restrict__ lmeta = nullptr) {
    typedef typename VecT<E, VEC>::type Vt;
    const int lane = (int)lane_id();
    const int64_t r = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (r >= rows) return;
    const E *row = pmf + (t0 + r / B) * step_stride + (r % B) * stream_stride;
    constexpr bool W = sizeof(E) == 8;
    const int64_t nvec = V / VEC, nit = (nvec + 63) / 64, ngrp = (nit + 7) / 8;
    int64_t CI, nch;
    dec_chunk_layout<E, VEC>(V, &CI, &nch);
    uint64_t mine = 0;
    E mn = (E)~(E)0;
    uint32_t ovf = 0;
    // groups of 8 iterations (8 loads in flight per lane), their 8 totals from one
    // butterfly, each added into the lane of its chunk (chunk = iteration / CI); LEAN u64
    // rows also into the lane of their lean chunk (lean_chunk_layout), chunks 64.. in lmB
    int64_t chunk = 0, left = CI;
    int64_t LCI = CI, lnch = nch;
    if constexpr (LEAN && LeanCW<E> == 2) lean_chunk_layout<E, VEC>(V, &LCI, &lnch);
    int64_t lch = 0, lleft = LCI;
    uint64_t lmA = 0, lmB = 0;
    E run = 0;                                                 // LEAN: the row's sum so far
    Vt *cp = LEAN ? reinterpret_cast<Vt *>(lcdf + r * V) : nullptr;
    // LEAN: a group's CDF vectors are stored after the next group's loads are issued, so
    // the in-order wait for those loads never waits on these stores
    Vt pv[8];
    int64_t pg = -1;
    auto store_pending = [&]() {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int64_t vi = (pg * 8 + u) * 64 + lane;
            if (vi < nvec) cp[vi] = pv[u];
        }
    };
    for (int64_t g = 0; g < ngrp; g++) {
        Vt x[8];
#pragma unroll
        for (int u = 0; u < 8; u++) x[u] = load_vec_or0<E, VEC>(row, (g * 8 + u) * 64 + lane, nvec);
        if constexpr (LEAN) {
            __builtin_amdgcn_sched_barrier(0);
            if (pg >= 0) store_pending();
        }
        uint64_t s8[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            uint64_t a = 0;
#pragma unroll
            for (int j = 0; j < VEC; j++) {
                const E e = vget<E, VEC>(x[u], j);
                a = add_ovf<W>(a, (uint64_t)e, ovf);
                const E m1 = e - 1;
                mn = m1 < mn ? m1 : mn;
            }
            s8[u] = a;
        }
        if constexpr (LEAN && VEC > 1) {
#pragma unroll
            for (int u = 0; u < 8; u++) {
                E in, tot;
                if constexpr (W) {
                    in = wave_incl_scan_u64(s8[u]);
                    tot = readlane_u64(in, 63);
                } else {
                    in = wave_incl_scan_u32((uint32_t)s8[u]);
                    tot = (uint32_t)__builtin_amdgcn_readlane((int)in, 63);
                }
                E c = run + in - (E)s8[u];                     // the row's sum before this lane's entries
                Vt cv;
#pragma unroll
                for (int j = 0; j < VEC; j++) {
                    c += vget<E, VEC>(x[u], j);
                    cv[j] = c;
                }
                pv[u] = cv;
                run += tot;
            }
            pg = g;
        }
        const uint64_t tot = wave_sum8_u64<W>(s8, ovf);       // lane l: iteration g*8 + (l & 7)
#pragma unroll
        for (int u = 0; u < 8; u++) {
            if (g * 8 + u >= nit) break;
            const uint64_t v = readlane_u64(tot, u);
            if (lane == chunk) mine = add_ovf<W>(mine, v, ovf);
            if (--left == 0) { chunk++; left = CI; }
            if constexpr (LEAN && LeanCW<E> == 2) {
                if (lane == (lch & 63)) {
                    if (lch < 64) lmA += v;
                    else lmB += v;
                }
                if (--lleft == 0) { lch++; lleft = LCI; }
            }
        }
    }
    if constexpr (LEAN) {
        if (pg >= 0) store_pending();
    }
    uint64_t minp;
    if constexpr (sizeof(E) == 8) minp = wave_min_u64(mn) + 1;
    else minp = (uint64_t)wave_min_u32(mn) + 1;
    const u128 acc128 = wave_sum_u128((u128)mine);
    const bool bad = __any(ovf) || (acc128 >> 64) || acc128 == 0;
    chunks[r * 64 + lane] = mine;
    if (lane == 0) meta[r] = DecRowMeta{bad ? 0 : (uint64_t)acc128, minp};
    if constexpr (LEAN) {
        const uint64_t in = wave_incl_scan_u64(mine);
        const uint64_t T = (uint64_t)acc128;
        const bool ok = !bad && lean_total_ok<E>(T) && minp != 0;
        // chunk lane's exclusive bound; a row not for the lean step gets bounds no target
        // passes (c*w <= v*T fails for c = 2^64 - 1 and for its low word), so the step finds
        // no chunk and leaves without testing T
        if constexpr (LeanCW<E> == 2) {
            const uint64_t ia = wave_incl_scan_u64(lmA), ib = wave_incl_scan_u64(lmB) + readlane_u64(ia, 63);
            u64x2 bnd;
            bnd.x = ok ? ia - lmA : ~0ull;
            bnd.y = ok ? ib - lmB : ~0ull;
            reinterpret_cast<u64x2 *>(lchunk)[r * 64 + lane] = bnd;
        } else {
            lchunk[r * 64 + lane] = ok ? in - mine : ~0ull;
        }
        // 1/T correctly rounded (an IEEE divide, once per row): the one-estimate bounds of
        // div_mid (u64 rows) and div_near (u32 rows) need it
        if (lane == 0)
            lmeta[r] = LeanMeta{ok ? T : 0, ok ? (T + minp - 1) / minp : 0, 1.0 / (double)(ok ? T : 1), (double)T};
    }
}

template <typename E, int VEC>
// No occupancy bound: it runs one wave per stream for few streams (the stats path), where the
// serial chain, not residency, sets the pace; the 4-waves/SIMD cap spilled the u64 form.
__global__ __launch_bounds__(256) void k_decode_seq(const E *__restrict__ pmf, int64_t step_stride, int64_t stream_stride,
                                            int64_t t0, int64_t nsteps, int64_t V, int prec,
                                            const uint64_t *__restrict__ chunks,
                                            const DecRowMeta *__restrict__ meta, DecState *states,
                                            const uint8_t *bits, uint64_t stride, const uint64_t *nbits,
                                            int32_t *sym_out, int64_t B, int mapping,
                                            int64_t *__restrict__ resume = nullptr, int64_t rstep = -1,
                                            int stop_undet = 0, int64_t max_steps = INT64_MAX) {
    const int lane = (int)lane_id();
    // rows of statistics per step: B, or 0 for a static model (stride-0 steps: one row per stream)
    if (rstep < 0) rstep = B;
    // the stream index and its decoder state wave-uniform (SGPRs): the serial chain --
    // the targets, the ranges, the renormalisation -- then runs on the scalar unit
    // (decode_symbol<..., true>), with uniform branches instead of exec-masked ones
    const int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + wave_in_block();
    if (b >= B) return;
    DecState st = states[b];
    dec_state_uniform(st);
    const uint8_t *mybits = bits + b * stride;
    const uint64_t mynbits = nbits[b];
    int64_t CI, nch;
    dec_chunk_layout<E, VEC>(V, &CI, &nch);
    // after k_decode_lean: its steps are done, continue from the first it left
    const int64_t i0 = resume ? (int64_t)rfl_u64((uint64_t)(resume[b] - t0)) : 0;
    if (i0 >= nsteps) return;
    // max_steps: only that many -- the step a lean launch left at; resume[b] then moves past
    // them and the next lean launch goes on from there
    const int64_t iend = max_steps < nsteps - i0 ? i0 + max_steps : nsteps;
    uint64_t next = chunks[(i0 * rstep + b) * 64 + lane];
    DecRowMeta nmeta = meta[i0 * rstep + b];
#if LAC_DEC_PHASES
    PhaseClock clock, *clk = &clock;
    clock.start();
#else
    NoClock *clk = nullptr;
#endif
    for (int64_t i = i0; i < iend; i++) {
        dec_state_uniform(st);                                 // (the loop's phis are not seen as uniform)
        const int64_t t = t0 + i;
        const uint64_t mine = next;
        const DecRowMeta rm = nmeta;
        if (i + 1 < iend) {                                    // prefetch: independent of the state
            next = chunks[((i + 1) * rstep + b) * 64 + lane];
            nmeta = meta[(i + 1) * rstep + b];
        }
        int32_t *out = sym_out + t * B + b;
        if (st.err) {                                          // failed or stopped: -1 for the rest, 64 at once
            for (int64_t j = i + lane; j < nsteps; j += 64) sym_out[(t0 + j) * B + b] = -1;
            break;
        }
        const E *row = pmf + t * step_stride + b * stream_stride;
        int err = rm.T ? 0 : LAC_E_TABLE;
        int64_t s = -1;
        if (!err) {
            const uint64_t incl = wave_incl_scan_u64(mine);
            auto find_chunk = [&](uint64_t tgt, int64_t *cv0, int *g, uint64_t *cb) {
                const uint64_t ex = incl - mine;
                const bool hit = lane < nch && ex <= tgt && tgt < incl;
                const uint64_t mask = __ballot(hit);
                if (!mask) return false;
                const int src = __ffsll((unsigned long long)mask) - 1;
                *cv0 = (int64_t)src * CI * 64;
                *g = (int)CI;
                *cb = readlane_u64(ex, src);
                return true;
            };
            if (clk) clk->mark(0);
            err = decode_symbol<E, VEC, decltype(find_chunk), true>(st, row, V, rfl_u64(rm.T), rfl_u64(rm.minp), prec,
                                                                   mapping, mybits, mynbits, find_chunk, &s, clk,
                                                                   NoIdle(), stop_undet != 0);
        }
        if (err) {
            st.err = err;
            st.err_step = st.nsym;
        }
        if (lane == 0) *out = err ? -1 : (int32_t)s;
    }
    if (lane == 0) states[b] = st;
    if (max_steps != INT64_MAX && lane == 0) resume[b] = t0 + iend;
#if LAC_DEC_PHASES
    if (lane == 0) {
        for (int k = 0; k < 6; k++) atomicAdd(&g_dec_phase[k], (unsigned long long)clock.acc[k]);
        atomicAdd(&g_dec_phase[6], (unsigned long long)nsteps);
    }
#endif
}

// ---- lean few-stream decode step (stats path, prec <= 50)
// k_decode_seq's serial step for what few-stream decodes nearly always are -- u32 tables
// with totals below 2^32 and u64 tables of any valid total (llama-scale tables near 2^60,
// the drop-in surface's static tables), an unfudged range (or the floor mapping), prec
// <= 50 -- laid out for the latency of one wave, whose instructions issue in order.
// Everything that depends on the row alone comes precomputed from k_dec_stats<..., LEAN>:
// the row's per-entry CDF, the chunks' exclusive bounds, T's reciprocal and the fudge
// threshold ceil(T/minp), the bounds and thresholds loaded two steps ahead.  Left on the
// chain: a ballot over the chunk bounds compared with the target floor(v*T/w) as products
// (ex*w <= v*T, no division: the chunk is the last one whose bound passes), one round of
// loads of the chunk's CDF vectors (one 16-B vector per lane and iteration) with the
// target's division in its shadow, the iteration by the CDF value just before it, a ballot
// over the lanes' last entries, the two range divisions and the renormalisation.  Symbols
// collect one per lane and leave in one store per 64 steps.
// Results are k_decode_seq's.  A step outside the case (a bad, large or fudged row, an
// inconsistent state or stream) -- or, with LAC_OPT_DECODE_STOP, a symbol the bits do not
// determine -- ends this kernel for its stream before the step changes anything:
// resume[b] holds the step and k_decode_seq continues from it, raising the error (or
// stopping) there.  One wave per workgroup: streams spread over the XCDs.
// rstep: rows of statistics per step, B -- or 0 for a static model (stride-0 steps), whose
// one row per stream every step reads (L2-resident after the first).
// Few-stream lean decode: the re-read of step i's chunk is one dependent load per step,
// an HBM round trip when the row is cold.  Helper waves -- workgroups of the same launch
// placed on the decoding wave's XCD (workgroups are dealt to the 8 XCDs round-robin, so
// index = stream mod 8) -- read one dword of every 128-B line of the CDF rows a few steps
// ahead of the decoder, which then finds its chunk in that XCD's L2.  They only read: the
// values are discarded (an empty asm consumes them so the loads stay).  They pace
// themselves by the decoder's progress (a relaxed agent-scope counter it sets every 8
// steps), never the other way round: results do not depend on them, and a helper that
// sees no progress for ~10 ms gives up, so the grid always drains.
#ifndef LAC_LEAN_AHEAD
#define LAC_LEAN_AHEAD 16
#endif
#ifndef LAC_LEAN_HELPERS
#define LAC_LEAN_HELPERS 16
#endif
constexpr int kLeanAhead = LAC_LEAN_AHEAD;      // rows prefetched ahead of the decoder
constexpr int kLeanHelpers = LAC_LEAN_HELPERS;  // helper waves per stream
// Up to 44 streams: the stats pass of the lean step writes a full CDF copy of every row, so
// its per-step cost grows with the streams, and k_decode_seq's read-only pass overtakes it
// between 32 and 64 (V=32000 u32, decode us per step lean / seq: 8 streams 1.17 / 2.75,
// 16 1.76 / 2.90, 32 2.75 / 3.25, 64 4.52 / 3.91; profiles/r06/lean3/fewstreams/)
#ifndef LAC_LEAN_MAX_STREAMS
#define LAC_LEAN_MAX_STREAMS 44
#endif
constexpr int64_t kLeanMaxStreams = LAC_LEAN_MAX_STREAMS;   // k_decode_lean up to this many streams
constexpr int kLeanHelpMaxStreams = 16;         // above: no helpers (L2: ~2.6 MB ahead per stream)
#ifndef LAC_LEAN_PUB
#define LAC_LEAN_PUB 8
#endif
constexpr int kLeanPub = LAC_LEAN_PUB;          // the decoder publishes its progress every kLeanPub steps
#ifndef LAC_LEAN_BYTES
#define LAC_LEAN_BYTES (512ll << 20)   // (256 MB: c2 u64 1.47 us per step, 512 MB 1.44: more stats waves per CU)
#endif
constexpr int64_t kLeanBytes = LAC_LEAN_BYTES;  // CDF rows per launch: at most this many bytes
#ifndef LAC_LEAN_ROUNDS
#define LAC_LEAN_ROUNDS 3
#endif
constexpr int kLeanRounds = LAC_LEAN_ROUNDS;    // k_decode_seq one step + lean again, per launch group
#ifndef LAC_LEAN_WIDE_WINDOW
#define LAC_LEAN_WIDE_WINDOW 1                  // wide u64 rows: the search against a double window
#endif

__device__ inline int32_t lean_progress(const int32_t *p) {
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

__device__ inline void lean_touch(const uint8_t *base, int64_t bytes) {
    // one dword of every 128-B line of [base, base + bytes), 16 loads in flight per lane
    if (bytes < 4) return;
    const int64_t lines = (bytes - 4) / 128 + 1;
    for (int64_t l0 = 0; l0 < lines; l0 += 16 * 64) {
        uint32_t v[16];
#pragma unroll
        for (int u = 0; u < 16; u++) {
            const int64_t ln = l0 + u * 64 + (int64_t)lane_id(), lc = ln < lines ? ln : lines - 1;
            v[u] = *reinterpret_cast<const uint32_t *>(base + lc * 128);
        }
#pragma unroll
        for (int u = 0; u < 16; u++) asm volatile("" ::"v"(v[u]));   // (prefetch only: the value is unused)
    }
}

template <typename E>
__device__ void lean_helper(const E *lcdf, const uint64_t *lchunk, const LeanMeta *lmeta, int64_t rstep, int32_t n32,
                            int64_t V, int64_t B, int64_t B8, const int32_t *progress) {
    const int64_t hidx = (int64_t)blockIdx.x - B8;
    const int64_t b = hidx % B8, k = hidx / B8;                 // stream (same XCD: B8 % 8 == 0), helper
    if (b >= B || k >= kLeanHelpers) return;
    int32_t seen = 0;
    for (int32_t t = (int32_t)k; t < n32; t += kLeanHelpers) {
        int64_t idle = 0;
        while (seen + kLeanAhead < t) {
            seen = lean_progress(progress + b);
            if (seen + kLeanAhead >= t) break;
            if (++idle > (1 << 17)) return;                      // ~10 ms without progress
            __builtin_amdgcn_s_sleep(2);
        }
        const int64_t r = (int64_t)t * rstep + b;
        lean_touch(reinterpret_cast<const uint8_t *>(lcdf + r * V), V * (int64_t)sizeof(E));
        // the row's chunk bounds and LeanMeta, which the decoder loads two steps ahead
        lean_touch(reinterpret_cast<const uint8_t *>(lchunk + r * 64 * LeanCW<E>), 64 * LeanCW<E> * (int64_t)sizeof(uint64_t));
        lean_touch(reinterpret_cast<const uint8_t *>(lmeta + r), (int64_t)sizeof(LeanMeta));
    }
}

// The bit streams as k_decode_lean reads them: word j of stream b holds stream bits
// 64j .. 64j+63 in reading order (the stream's 8 bytes byte-swapped), bits past nbits cleared,
// then zero words to the row's end (wstride = stride / 8 + 2 words per stream).  The step then
// reads its 128-bit window as two scalar words at one clamped index, with no end mask and no
// byte swaps on its chain.  Built once per decode call (the streams are constant while open).
__global__ __launch_bounds__(256) void k_lean_window(const uint8_t *__restrict__ bits, uint64_t stride,
                                                     const uint64_t *__restrict__ nbits, uint64_t *__restrict__ win,
                                                     int64_t wstride, int64_t B) {
    const int64_t b = blockIdx.y;
    if (b >= B) return;
    const uint64_t nb = nbits[b], cap = stride / 8;
    const uint64_t nw = (nb + 63) >> 6 < cap ? (nb + 63) >> 6 : cap;   // (nb > 8 * stride fails in k_dec_init)
    const uint64_t *src = reinterpret_cast<const uint64_t *>(bits + b * stride);
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < wstride; j += (int64_t)gridDim.x * 256) {
        uint64_t w = 0;
        if ((uint64_t)j < nw) {
            w = bswap64(src[j]);
            const uint64_t in = nb - (uint64_t)j * 64;         // stream bits in this word
            if (in < 64) w &= ~0ull << (64 - in);
        }
        win[b * wstride + j] = w;
    }
}

// e * w <= P (P = v * T as hi:lo): the chunk test of the lean step, lane-parallel.  u32 tables:
// e < 2^32, w < 2^51, the products split at bit 32 (below 2^83); u64 tables: e < 2^50, full
// 128-bit products (below 2^101).
template <typename E>
__device__ inline bool lean_le(uint64_t e, uint64_t wl, uint64_t wh, uint64_t w, uint64_t ph, uint64_t pl) {
    if constexpr (sizeof(E) == 4) {
        const uint64_t q0 = (e & 0xffffffffull) * wl, qh = (e & 0xffffffffull) * wh + (q0 >> 32);
        return (qh < ph) | ((qh == ph) & ((uint32_t)q0 <= (uint32_t)pl));
    } else {
        const u128 q = (u128)e * w;
        const uint64_t qh = (uint64_t)(q >> 64), ql = (uint64_t)q;
        return (qh < ph) | ((qh == ph) & (ql <= pl));
    }
}

template <typename E, int VEC, int CIM>
__global__ __launch_bounds__(64) void k_decode_lean(const E *__restrict__ lcdf, int64_t rstep, int64_t t0,
                                                    int64_t nsteps, int64_t V, int prec,
                                                    const uint64_t *__restrict__ lchunk,
                                                    const LeanMeta *__restrict__ lmeta, DecState *states,
                                                    const uint64_t *__restrict__ lwin, int64_t wstride,
                                                    const uint64_t *__restrict__ nbits, int32_t *sym_out, int64_t B,
                                                    int mapping, int stop_undet, int64_t *__restrict__ resume,
                                                    int32_t *progress, int restart) {
    typedef typename VecT<E, VEC>::type Vt;
    constexpr bool W = sizeof(E) == 8;
    const int lane = (int)lane_id();
    const int64_t B8 = (B + 7) & ~(int64_t)7;
    if ((int64_t)blockIdx.x >= B8) {                             // a helper workgroup
        if (progress) lean_helper<E>(lcdf, lchunk, lmeta, rstep, (int32_t)nsteps, V, B, B8, progress);
        return;
    }
    const int64_t b = blockIdx.x;
    if (b >= B) return;
    DecState st = states[b];
    dec_state_uniform(st);
    const uint64_t *mywin = lwin + b * wstride;
    const uint64_t mynbits = rfl_u64(nbits[b]);
    const uint64_t nwc = (uint64_t)wstride - 2;                 // words past the stream's own: zero
    const uint64_t mynw = (mynbits + 63) >> 6 < nwc ? (mynbits + 63) >> 6 : nwc;
    int64_t CI, nch;
    lean_chunk_layout<E, VEC>(V, &CI, &nch);
    const int32_t nv32 = (int32_t)(V / VEC);                    // (<= 32768: CI <= 4)
    const uint32_t ci64 = (uint32_t)CI * 64;
    const int32_t nch32 = (int32_t)nch;
    const bool ceil_map = mapping != LAC_MAP_FLOOR;
    // restart: a later launch over the same group, from the step after the one k_decode_seq
    // took for the stream (resume[b]); its steps and rows are counted from there
    const int32_t i0 = restart ? (int32_t)rfl_u64((uint64_t)(resume[b] - t0)) : 0;
    const int32_t n32 = (int32_t)nsteps - i0;                  // (<= the launch's steps)
    // row data two steps ahead: the lane's chunk bound (per-lane pointer) and the LeanMeta
    // (by index, a scalar load) in two register sets A / B that the 2x unrolled loop uses in
    // turn, so a prefetched value is first touched two steps after its load was issued (a
    // single set rotated by copies waited at the next step for a load issued one step
    // earlier); a static model (rstep 0) reloads its one row's.  A running pointer to row
    // i's CDF.
    // The LeanMeta arrives by a vector load (lane k: word k & 3), read out with readlanes:
    // a scalar load's wait (lgkmcnt, out of order) waits for every scalar load in flight,
    // so a row's meta two steps ahead was waited for one step after its load.
    const uint64_t *lmw = reinterpret_cast<const uint64_t *>(lmeta) + (lane & 3);
    // (unconditional -- the buffers hold two rows past a launch's last -- and drained here:
    // loads that differ between the loop's entry paths made the wait at its top a full drain
    // on every step)
    // (u64 rows: the lane's two chunk bounds, chunks lane and 64 + lane, as one 16-B vector)
    typedef typename std::conditional<LeanCW<E> == 2, u64x2, uint64_t>::type CWt;
    const CWt *lcw = reinterpret_cast<const CWt *>(lchunk);
    const int64_t r0 = (int64_t)i0 * rstep + b;                // this launch's first row
    CWt cwA = lcw[r0 * 64 + lane], cwB = lcw[(r0 + rstep) * 64 + lane];
    uint64_t lmA = lmw[r0 * 4], lmB = lmw[(r0 + rstep) * 4];
    __builtin_amdgcn_s_waitcnt(0);
    const CWt *lcv = lcw + (r0 + 2 * rstep) * 64 + lane;
    int64_t li = r0 + 2 * rstep;
    const Vt *rowp = reinterpret_cast<const Vt *>(lcdf + r0 * V);
    const int64_t rv_step = rstep * (int64_t)nv32;               // vectors per step
    int32_t *outv = sym_out + (t0 + i0 + lane) * B + b;         // lane j: step i0 + 64k + j
    // the registers as locals (SGPRs); the counters are settled after the loop
    int64_t l = st.l, h = st.h, x = st.x;
    uint64_t pos = st.pos;
    int32_t firstnd = -1;                                       // first step not determined
    int32_t sbuf = -1;
    int32_t i = 0;
#if LAC_DEC_PHASES
    PhaseClock clk;
    clk.start();
#else
    NoClock clk;
#endif
    // one step with row data (cwi, lm); the next-but-one row's loads go into (pcw, plm) once
    // this step's chunk loads are issued.  false: the stream leaves (not this step's case)
    // PUB: the first step of a pair, whose i is even, publishes the decoder's progress
    auto step = [&](const CWt cwi, const uint64_t lmv, CWt &pcw, uint64_t &plm, auto pub) -> bool {
        l = (int64_t)rfl_u64((uint64_t)l);                      // (the loop's phis are not seen as uniform)
        h = (int64_t)rfl_u64((uint64_t)h);
        x = (int64_t)rfl_u64((uint64_t)x);
        pos = rfl_u64(pos);
        const uint64_t T = readlane_u64(lmv, 0), fthr = readlane_u64(lmv, 1);   // LeanMeta {T, fthr, iT}
        const double iT = __builtin_bit_cast(double, readlane_u64(lmv, 2));
        const double Td = __builtin_bit_cast(double, readlane_u64(lmv, 3));
        const Vt *row = rowp;
        rowp += rv_step;
        const uint64_t w = (uint64_t)(h - l + 1), v = (uint64_t)(x - l);
        clk.mark(0);
        // the chunk holding tgt = floor(v*T/w) without the division: the last chunk whose
        // exclusive bound ex passes ex <= tgt, i.e. ex*w <= v*T (ex nondecreasing over the
        // chunks, and tgt < T, so that chunk's inclusive bound exceeds tgt)
        uint64_t ph, pl;
        if constexpr (W) {
            const u128 P = (u128)v * T;
            ph = rfl_u64((uint64_t)(P >> 64));
            pl = rfl_u64((uint64_t)P);
        } else {
            const uint64_t p0 = (v & 0xffffffffull) * T;
            ph = (v >> 32) * T + (p0 >> 32);
            pl = (uint32_t)p0;
        }
        const uint32_t wl = (uint32_t)w;
        const uint64_t wh = w >> 32;
        auto le = [&](uint64_t e) { return lean_le<E>(e, wl, wh, w, ph, pl); };   // e <= tgt
        uint64_t cm;
        uint32_t src;
        // the chunk's loads first (in bounds whatever the step: refused below if it is bad),
        // then the stream window, then the next-but-one row's data, then everything that
        // can wait for them
        if constexpr (LeanCW<E> == 2) {
            cm = __ballot((lane < nch32) & le(cwi.x));
            const uint64_t cm1 = __ballot((lane + 64 < nch32) & le(cwi.y));
            src = cm1 ? 127u - (uint32_t)__builtin_clzll((unsigned long long)cm1)
                      : cm ? (uint32_t)(63 - __builtin_clzll((unsigned long long)cm)) : 0u;
        } else {
            cm = __ballot((lane < nch32) & le(cwi));
            src = cm ? (uint32_t)(63 - __builtin_clzll((unsigned long long)cm)) : 0u;
        }
        const int32_t cv0 = (int32_t)(src * ci64);
        Vt xs[CIM];
#pragma unroll
        for (int g = 0; g < CIM; g++) {
            const int32_t vi = cv0 + g * 64 + lane, vc = vi < nv32 ? vi : nv32 - 1;
            xs[g] = row[vc];
        }
        // the stream window: words pos/64 and the next, clamped to the zero words past the end
        const uint64_t wi = (pos >> 6) < mynw ? (pos >> 6) : mynw;
        const uint64_t W0 = mywin[wi], W1 = mywin[wi + 1];
        // row i+2 (the buffers hold two rows past the launch's last: read, never used); a
        // static model reloads its one row.  Unconditional: under a branch the two paths'
        // load counts differ, and the wait for this step's chunk vectors then also waited
        // for these loads (from HBM) on the moving path.
        pcw = *lcv;
        plm = lmw[li * 4];
        lcv += rstep * 64;
        li += rstep;
        if constexpr (decltype(pub)::value) {
            if (__builtin_expect(progress && (i & (kLeanPub - 1)) == 0, 0) && lane == 0)   // the helpers' pace
                __hip_atomic_store(progress + b, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // (after the loads)
        }
        // a step outside the lean case leaves at the end (a branch here would let the
        // compiler sink the loads below it); until then its divisions run on safe values
        // (the step's tests as sign bits of differences and ORs on the scalar unit, one
        // exit test per step)
        // (a row not for the lean step, T = 0 in its LeanMeta, has chunk bounds no target passes: cm == 0)
        // (unsigned differences: signed ones were folded back into ordered 64-bit compares,
        // which are vector instructions)
        const uint64_t bad = (((uint64_t)x - (uint64_t)l) >> 63) | (((uint64_t)h - (uint64_t)x) >> 63) |
                             ((uint64_t)ceil_map & ((w - fthr) >> 63)) | (uint64_t)(cm == 0);
        // (a bad step computes on whatever values it has -- no load or store depends on them
        // -- and leaves at the exit test below)
        const uint64_t Ts = T, ws = w, vs = v;
        uint64_t ex0;
        if constexpr (LeanCW<E> == 2) ex0 = readlane_u64(src >= 64 ? cwi.y : cwi.x, (int)(src & 63));
        else ex0 = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)cwi, (int)src);
        // the target: u32 rows and u64 rows below 2^50 divide (div_small, in the loads'
        // shadow) and compare entries with it; u64 rows of 2^50 and more (llama-scale
        // tables), whose target would divide in 128 bits past the loads' return, compare
        // entries by products (c*w <= v*T) and take div_mid's ranges
        const bool small = !W || Ts < kSmallQuot;               // uniform
        // (div_near: the estimate is within one of the quotient, two sign tests; for u64 rows,
        // whose target reaches 2^50, with 1/w to ~1 ulp)
        const double iw = W ? recip2_small(ws) : recip_small(ws);   // (w <= 2^50: exact as a double)
        // (u64 rows of 2^50 and more: no exact target -- by div_floor_inv's two estimates and
        // 128-bit remainders in the loads' shadow it measured slower, 1.775 vs 1.70 us per c2
        // step, profiles/r06/lean/ -- but the window below: 1.418 vs 1.442 us with products
        // alone, profiles/r06/lean3/widewindow/)
        const E te = (!W || small) ? (E)div_near_u(vs, Ts, 0, ws, iw) : (E)0;
        // u64 rows of 2^50 and more: a window [tlo, thi] around v*T/w from doubles that holds
        // the target -- v exact, T within an ulp, 1/w to ~2^-50 (one Newton step), so the
        // estimate is within 2^15 of v*T/w < 2^64 -- with 2^16 of margin either side.  The
        // search compares entries with tlo; it equals the exact search unless a compared entry
        // lies in (tlo, thi], which one ballot tests (then the search reruns with products).
        uint64_t tlo = 0, thi = 0;
        if constexpr (W) {
            if (!small) {
                const double lo_d = small_to_f64(vs) * Td * recip_small(ws) - 65536.0;
                tlo = rfl_u64(lo_d > 0.0 ? (uint64_t)lo_d : 0);
                thi = tlo > ~0ull - 131072 ? ~0ull : tlo + 131072;
            }
        }
        clk.mark(1);
        clk.mark(2);
        int gs = 0;
        E exg = (E)ex0;
        uint64_t m2, lo_l, hi_c, prev;
        uint32_t kL;
        int L;
        Vt xgo;                                                 // the iteration's vectors the search took
        auto search = [&](auto lte) {                           // lte(c): c <= tgt
            // the iteration holding the target: the last whose CDF value just before it (the
            // chunk's bound, else lane 63's last entry of the iteration before) is <= tgt.
            // (Its vectors selected by the take tests themselves: a select on gs == g was
            // turned into an indexed read of xs[] through scratch memory for CIM >= 3.)
            Vt xg = xs[0];
#pragma unroll
            for (int g = 1; g < CIM; g++) {
                const E eg = W ? (E)readlane_u64((uint64_t)vget<E, VEC>(xs[g - 1], VEC - 1), 63)
                               : (E)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)vget<E, VEC>(xs[g - 1], VEC - 1), 63);
                const bool take = (cv0 + g * 64 < nv32) & lte(eg);
                gs = take ? g : gs;
                exg = take ? eg : exg;
                xg = take ? xs[g] : xg;
            }
            xgo = xg;
            const bool real = cv0 + gs * 64 + lane < nv32;
            m2 = __ballot(real & !lte(vget<E, VEC>(xg, VEC - 1)));
            L = m2 ? __ffsll((unsigned long long)m2) - 1 : 0;
            // lane L's entries: k of them <= tgt, then the symbol's; its lower bound is the
            // entry before (lane L's, lane L-1's last, or the iteration's start value)
            uint32_t k = 0;
            E lo = 0, hi = vget<E, VEC>(xg, VEC - 1);
#pragma unroll
            for (int j = VEC - 1; j >= 0; j--) {
                const E c = vget<E, VEC>(xg, j);
                const bool cle = lte(c);
                k += cle ? 1 : 0;
                hi = cle ? hi : c;
                lo = (cle && lo == 0) ? c : lo;                 // the last entry <= tgt (entries ascend)
            }
            const int Lp = L > 0 ? L - 1 : 0;
            if constexpr (W) {
                lo_l = readlane_u64(lo, L);
                hi_c = readlane_u64(hi, L);
                prev = readlane_u64(vget<E, VEC>(xg, VEC - 1), Lp);
            } else {
                lo_l = (uint32_t)__builtin_amdgcn_readlane((int)lo, L);
                hi_c = (uint32_t)__builtin_amdgcn_readlane((int)hi, L);
                prev = (uint32_t)__builtin_amdgcn_readlane((int)vget<E, VEC>(xg, VEC - 1), Lp);
            }
            kL = (uint32_t)__builtin_amdgcn_readlane((int)k, L);
        };
        if (!W || small) search([&](E c) { return c <= te; });
        else if (!LAC_LEAN_WIDE_WINDOW) search([&](E c) { return le((uint64_t)c); });
        else {
            search([&](E c) { return (uint64_t)c <= tlo; });
            auto inw = [&](uint64_t c) { return (c > tlo) & (c <= thi); };
            bool amb = false;
#pragma unroll
            for (int g = 1; g < CIM; g++)
                amb |= inw(readlane_u64((uint64_t)vget<E, VEC>(xs[g - 1], VEC - 1), 63));
            bool la = false;
#pragma unroll
            for (int j = 0; j < VEC; j++) la |= inw((uint64_t)vget<E, VEC>(xgo, j));
            if (__builtin_expect(amb | (__ballot(la) != 0), 0)) {
                gs = 0;
                exg = (E)ex0;
                search([&](E c) { return le((uint64_t)c); });
            }
        }
        const uint64_t lo_c = kL ? lo_l : (L > 0 ? prev : (uint64_t)exg);
        const int32_t sym = (cv0 + gs * 64 + L) * VEC + (int32_t)kL;
        clk.mark(3);
        uint64_t a, bb;
        if (!W) div_near_u2<true>(lo_c, hi_c, ws, ceil_map ? Ts - 1 : 0, Ts, iT, &a, &bb);
        else if (small) div_near_u2<false>(lo_c, hi_c, ws, ceil_map ? Ts - 1 : 0, Ts, iT, &a, &bb);
        else div_mid_u2(lo_c, hi_c, ws, ceil_map ? Ts - 1 : 0, ceil_map ? Td : 0.0, Ts, iT, &a, &bb);
        // (l + a <= x <= l + bb - 1: v in [a, bb))
        if (bad | (uint64_t)(m2 == 0) | ((vs - a) >> 63) | (((vs - bb) >> 63) ^ 1)) return false;
        clk.mark(4);
        // the 1-padded end past the stream's end (u > 0; before it the step is determined):
        // determined iff vhi < w and floor(vhi*T/w) < hi_c, i.e. vhi*T < hi_c*w
        if (__builtin_expect((mynbits - pos) >> 63, 0)) {        // pos > nbits
            const uint64_t past = pos - mynbits;
            const int u = past < (uint64_t)prec ? (int)past : prec;
            const uint64_t vhi = vs + ((1ull << u) - 1);
            const bool vhi_in = (vhi - ws) >> 63;                 // vhi < w
            const u128 PH = (u128)vhi * Ts, HW = (u128)hi_c * ws;
            if (!(vhi_in && PH < HW)) {                           // not determined
                if (stop_undet) return false;                     // k_decode_seq stops the stream here
                if (firstnd < 0) firstnd = i;
            }
        }
        // narrow + renormalise (decode_advance<true>) without branches: kk = 0 keeps the
        // registers and reads no window bits
        int64_t nl = l + (int64_t)a, nh = l + (int64_t)bb - 1;
        const uint64_t d = (uint64_t)(nh - nl);
        const int sh = bitlen64(d), kk0 = prec - sh, kk = kk0 > 0 ? kk0 : 0;   // (renorm: kk <= 0 is 0)
        const uint64_t Ev = kk > 0 ? (uint64_t)nl >> sh : 0;
        nl = (int64_t)(((uint64_t)nl - (Ev << (sh & 63))) << kk);
        nh = nl + (int64_t)((d + 1) << kk) - 1;
        // the top kk bits of the window at pos (kk <= 50; bits past the stream's end are zeros)
        const int off = (int)(pos & 63);
        const uint64_t W0u = rfl_u64(W0), W1u = rfl_u64(W1);
        const uint64_t wv = (((W0u << off) | ((W1u >> 1) >> (63 - off))) >> 1) >> (63 - kk);
        x = (int64_t)((((uint64_t)x - (Ev << (sh & 63))) << kk) | wv);
        pos += (uint64_t)kk;
        l = nl;
        h = nh;
        if (lane == (i & 63)) sbuf = sym;
        if (__builtin_expect((i & 63) == 63, 0)) {
            *outv = sbuf;
            outv += B * 64;
        }
        clk.mark(5);
        return true;
    };
    if (!st.err) {
        for (;;) {
            if (i >= n32 || !step(cwA, lmA, cwA, lmA, std::true_type{})) break;
            i++;
            if (i >= n32 || !step(cwB, lmB, cwB, lmB, std::false_type{})) break;
            i++;
        }
    }
#if LAC_DEC_PHASES
    if (lane == 0) {
        for (int k = 0; k < 6; k++) atomicAdd(&g_dec_phase[k], (unsigned long long)clk.acc[k]);
        atomicAdd(&g_dec_phase[6], (unsigned long long)i);
    }
#endif
    if (lane < (i & 63)) *outv = sbuf;
    if (progress && lane == 0)                                  // let the helpers go
        __hip_atomic_store(progress + b, 1 << 30, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lane == 0) {
        // the counters of decode_symbol for the i steps done
        if (st.det) {
            st.ndet += firstnd < 0 ? i : firstnd;
            st.det = firstnd < 0;
        }
        st.nsym += i;
        st.l = l;
        st.h = h;
        st.x = x;
        st.pos = pos;
        states[b] = st;
        resume[b] = t0 + i0 + i;
    }
}


#include "lac_tail.h"

}  // namespace

template <typename E, int VEC, int G>
static int decode_launch(lac_ctx *c, const E *pmf, int64_t step_off, int64_t stream_stride, int32_t *out,
                         hipStream_t st) {
    constexpr int64_t CH = 64 * VEC * G;
    const int64_t nch = (c->V + CH - 1) / CH;
    const size_t lds = sizeof(uint64_t) * (size_t)nch;
    if (lds > 64 * 1024) return fail(LAC_E_ARG, "vocab too large for the decode chunk table");
    ProfScope ps(c, KID_DECODE, st);
    if (c->B <= 256)        // few streams: 16 waves per stream keep the whole row in flight
        k_decode_step<E, VEC, G, 16><<<(unsigned)c->B, 64 * 16, lds, st>>>(
            pmf, step_off, stream_stride, c->V, c->prec, c->dec, c->dbits, c->dstride, c->dnbits, out, c->B,
            c->mapping);
    else
        k_decode_step<E, VEC, G, kWavesPerBlock><<<(unsigned)c->B, 64 * kWavesPerBlock, lds, st>>>(
            pmf, step_off, stream_stride, c->V, c->prec, c->dec, c->dbits, c->dstride, c->dnbits, out, c->B,
            c->mapping);
    CHECK_LAUNCH();
    return LAC_OK;
}

template <typename E, int VEC>
static int decode_wave_launch(lac_ctx *c, const E *pmf, int64_t step_stride, int64_t stream_stride, int64_t steps,
                              int32_t *out, hipStream_t st) {
    ProfScope ps(c, KID_DECODE_WAVE, st);
    const unsigned blocks = (unsigned)((c->B + kStreamWaves - 1) / kStreamWaves);
    const int64_t nit = (c->V / VEC + 63) / 64;               // 64-vector iterations per row
#define LAC_FINE(NR)                                                                                              \
    k_decode_wave_fine<E, VEC, NR><<<blocks, 64 * kStreamWaves, 0, st>>>(                                        \
        pmf, step_stride, stream_stride, steps, c->V, c->prec, c->dec, c->dbits, c->dstride, c->dnbits, out, c->B, \
        c->mapping)
    bool fine = false;
    if constexpr (VEC > 1) {
        fine = c->fine_decode && nit <= 512;
        if (fine && nit <= 128) LAC_FINE(2);
        else if (fine && nit <= 256) LAC_FINE(4);
        else if (fine) LAC_FINE(8);
    }
    if (!fine)
        k_decode_wave<E, VEC><<<blocks, 64 * kStreamWaves, 0, st>>>(
            pmf, step_stride, stream_stride, steps, c->V, c->prec, c->dec, c->dbits, c->dstride, c->dnbits, out, c->B,
            c->mapping);
#undef LAC_FINE
    CHECK_LAUNCH();
    return LAC_OK;
}

int ensure_chunk_buffers(lac_ctx *c) {
    if (!c->q1chunks) HIPCHK(hipMalloc(&c->q1chunks, sizeof(uint64_t) * 64 * c->chunk_steps * c->B));
    if (!c->q1m) HIPCHK(hipMalloc(&c->q1m, sizeof(float) * c->chunk_steps * c->B));
    if (!c->dmeta) HIPCHK(hipMalloc(&c->dmeta, sizeof(DecRowMeta) * c->chunk_steps * c->B));
    return LAC_OK;
}

template <typename E, int VEC>
static int decode_stats_path(lac_ctx *c, const E *pmf, int64_t step_stride, int64_t stream_stride, int64_t steps,
                             int32_t *out, hipStream_t st) {
    int rc = ensure_chunk_buffers(c);
    if (rc) return rc;
    const unsigned blocks = (unsigned)((c->B + kWavesPerBlock - 1) / kWavesPerBlock);
    // A static model (stride-0 steps): every step reads the same row per stream, so the
    // statistics are computed once per stream (rstep 0) and one launch pair covers any
    // number of steps.
    const bool stat = step_stride == 0;
    const int64_t rstep = stat ? 0 : c->B;
    // k_decode_lean: prec <= 50, chunks of at most 4 iterations (V <= 65536 entries: 64 chunk
    // bounds per u32 row, 128 per u64 row), totals lean_total_ok<E> (checked per row); its
    // CDF buffer holds up to kLeanBytes, so a launch takes at most that many steps' rows
    const int64_t nvec = c->V / VEC;
    int64_t CI, lnch;
    lean_chunk_layout<E, VEC>(c->V, &CI, &lnch);
    // Only for the fewest streams: the stats pass writes as many bytes more as it reads (the
    // CDF), which costs more than the shorter chain saves once enough streams run side by
    // side (round 4, per-vector CDF, V=32000: B=4 1.36 vs 2.66 us/step, 64 3.41 vs 3.96, 128
    // 5.39 vs 5.26; profiles/r04/lean/fewstreams/)
    const int64_t wstride = (int64_t)(c->dstride / 8) + 2;     // k_lean_window's words per stream
    bool lean = false;
    if constexpr (VEC > 1) lean = LAC_LEAN && c->prec <= 50 && CI <= 4 && nvec > 0 && c->B <= kLeanMaxStreams;
    int64_t cs = stat ? steps : c->chunk_steps;
    if (lean) {
        const int64_t rows_fit = kLeanBytes / (c->V * (int64_t)sizeof(E));
        if (!stat) {
            const int64_t fit = rows_fit / c->B;
            const int64_t ls = fit < 64 ? 64 : fit / 64 * 64;
            cs = ls < cs ? ls : cs;
        }
        const int64_t need = stat ? c->B : cs * c->B;          // CDF rows per launch
        if (c->lean_rows < need || c->lean_esize != (int)sizeof(E)) {
            (void)hipFree(c->lcdf);
            (void)hipFree(c->lchunk);
            (void)hipFree(c->lmeta);
            c->lcdf = nullptr;
            c->lchunk = nullptr;
            c->lmeta = nullptr;
            c->lean_rows = 0;
            HIPCHK(hipMalloc(&c->lcdf, sizeof(E) * need * c->V));
            // (two rows more: the step's prefetch of row i+2 reads past the launch's last row)
            HIPCHK(hipMalloc(&c->lchunk, sizeof(uint64_t) * 64 * LeanCW<E> * (need + 2 * c->B)));
            HIPCHK(hipMalloc(&c->lmeta, sizeof(LeanMeta) * (need + 2 * c->B)));
            c->lean_rows = need;
            c->lean_esize = (int)sizeof(E);
        }
        if (!c->dresume) HIPCHK(hipMalloc(&c->dresume, sizeof(int64_t) * c->B));
        const int64_t words = c->B * wstride;
        if (c->lwin_words < words) {
            (void)hipFree(c->lwin);
            c->lwin = nullptr;
            c->lwin_words = 0;
            HIPCHK(hipMalloc(&c->lwin, sizeof(uint64_t) * words));
            c->lwin_words = words;
        }
        const unsigned wblocks = (unsigned)((wstride + 255) / 256 < 64 ? (wstride + 255) / 256 : 64);
        k_lean_window<<<dim3(wblocks, (unsigned)c->B), 256, 0, st>>>(c->dbits, c->dstride, c->dnbits, c->lwin, wstride,
                                                                     c->B);
        CHECK_LAUNCH();
    }
    // prefetching helper workgroups for the fewest streams (kLeanHelpers per stream, dealt
    // to the stream's XCD); a static model's rows stay in L2 without them
    const bool help = lean && !stat && LAC_LEAN_HELP && c->B <= kLeanHelpMaxStreams;
    const int64_t B8 = (c->B + 7) & ~(int64_t)7;
    const unsigned lean_blocks = (unsigned)(help ? B8 * (1 + kLeanHelpers) : c->B);
    if (help && !c->dprogress) HIPCHK(hipMalloc(&c->dprogress, sizeof(int32_t) * c->B));
    for (int64_t t0 = 0; t0 < steps; t0 += cs) {
        const int64_t n = (steps - t0) < cs ? (steps - t0) : cs;
        const int64_t rows = stat ? c->B : n * c->B;
        ProfScope ps(c, KID_DECODE, st);
        const unsigned sblocks = (unsigned)((rows + kWavesPerBlock - 1) / kWavesPerBlock);
        // (a static model's statistics are computed by the first launch only)
        const bool fresh = !stat || t0 == 0;
        if constexpr (VEC > 1) {
            if (lean) {
                if (fresh) {
                    k_dec_stats<E, VEC, true><<<sblocks, 64 * kWavesPerBlock, 0, st>>>(
                        pmf, step_stride, stream_stride, c->B, rows, c->V, t0, c->q1chunks, (DecRowMeta *)c->dmeta,
                        (E *)c->lcdf, c->lchunk, (LeanMeta *)c->lmeta);
                    CHECK_LAUNCH();
                }
                if (help) HIPCHK(hipMemsetAsync(c->dprogress, 0, sizeof(int32_t) * c->B, st));
#define LAC_LEAN_K(CIM, NB, PROG, RESTART)                                                                      \
    k_decode_lean<E, VEC, CIM><<<NB, 64, 0, st>>>(                                                             \
        (const E *)c->lcdf, rstep, t0, n, c->V, c->prec, c->lchunk, (const LeanMeta *)c->lmeta, c->dec, c->lwin,   \
        wstride, c->dnbits, out, c->B, c->mapping, c->dec_stop, c->dresume, PROG, RESTART)
#define LAC_LEAN_SW(NB, PROG, RESTART)                                                                           \
    switch (CI) {                                                                                                \
    case 1: LAC_LEAN_K(1, NB, PROG, RESTART); break;                                                             \
    case 2: LAC_LEAN_K(2, NB, PROG, RESTART); break;                                                             \
    case 3: LAC_LEAN_K(3, NB, PROG, RESTART); break;                                                             \
    default: LAC_LEAN_K(4, NB, PROG, RESTART); break;                                                            \
    }
                LAC_LEAN_SW(lean_blocks, help ? c->dprogress : nullptr, 0);
                CHECK_LAUNCH();
                // a stream that left the lean step (a fudged range, a row outside the lean case)
                // gets that one step from k_decode_seq and the lean step again from the next,
                // kLeanRounds times; k_decode_seq then takes what is left.  A stream that did not
                // leave finds nothing to do in these launches.
                for (int k = 0; k < kLeanRounds; k++) {
                    k_decode_seq<E, VEC><<<blocks, 64 * kWavesPerBlock, 0, st>>>(
                        pmf, step_stride, stream_stride, t0, n, c->V, c->prec, c->q1chunks, (const DecRowMeta *)c->dmeta,
                        c->dec, c->dbits, c->dstride, c->dnbits, out, c->B, c->mapping, c->dresume, rstep, c->dec_stop, 1);
                    CHECK_LAUNCH();
                    LAC_LEAN_SW((unsigned)c->B, nullptr, 1);
                    CHECK_LAUNCH();
                }
#undef LAC_LEAN_SW
#undef LAC_LEAN_K
            }
        }
        if (!lean && fresh) {
            k_dec_stats<E, VEC><<<sblocks, 64 * kWavesPerBlock, 0, st>>>(
                pmf, step_stride, stream_stride, c->B, rows, c->V, t0, c->q1chunks, (DecRowMeta *)c->dmeta);
            CHECK_LAUNCH();
        }
        k_decode_seq<E, VEC><<<blocks, 64 * kWavesPerBlock, 0, st>>>(
            pmf, step_stride, stream_stride, t0, n, c->V, c->prec, c->q1chunks, (const DecRowMeta *)c->dmeta, c->dec,
            c->dbits, c->dstride, c->dnbits, out, c->B, c->mapping, lean ? c->dresume : nullptr, rstep, c->dec_stop);
        CHECK_LAUNCH();
    }
    return LAC_OK;
}

template <typename E, int VEC>
static int decode_block_launch(lac_ctx *c, const E *pmf, int64_t step_stride, int64_t stream_stride, int64_t steps,
                               int32_t *out, hipStream_t st) {
    ProfScope ps(c, KID_DECODE_WAVE, st);
    const int nw = c->block_waves ? c->block_waves : (c->B >= 1024 ? 4 : c->B >= 512 ? 8 : 16);
#define LAC_BLK(NW)                                                                                              \
    k_decode_block<E, VEC, NW><<<(unsigned)c->B, 64 * NW, 0, st>>>(pmf, step_stride, stream_stride, steps, c->V,  \
                                                                  c->prec, c->dec, c->dbits, c->dstride, c->dnbits, \
                                                                  out, c->B, c->mapping)
    if (nw == 4) LAC_BLK(4);
    else if (nw == 8) LAC_BLK(8);
    else LAC_BLK(16);
#undef LAC_BLK
    CHECK_LAUNCH();
    return LAC_OK;
}

static int decode_dispatch(lac_ctx *c, const void *pmf, int64_t step_stride, int64_t stream_stride, int64_t steps,
                           int32_t *out, hipStream_t st) {
    const uintptr_t p = (uintptr_t)pmf;
    if (c->dec_stop) {                      // LAC_OPT_DECODE_STOP: the stats path's kernels implement it
        if (c->pmf_bits == 32)
            return (p % 16 == 0) && c->V % 4 == 0 && step_stride % 4 == 0 && stream_stride % 4 == 0
                       ? decode_stats_path<uint32_t, 4>(c, (const uint32_t *)pmf, step_stride, stream_stride, steps, out, st)
                       : decode_stats_path<uint32_t, 1>(c, (const uint32_t *)pmf, step_stride, stream_stride, steps, out, st);
        return (p % 16 == 0) && c->V % 2 == 0 && step_stride % 2 == 0 && stream_stride % 2 == 0
                   ? decode_stats_path<uint64_t, 2>(c, (const uint64_t *)pmf, step_stride, stream_stride, steps, out, st)
                   : decode_stats_path<uint64_t, 1>(c, (const uint64_t *)pmf, step_stride, stream_stride, steps, out, st);
    }
    const bool wave = c->dpath == LAC_PATH_FUSED || (c->dpath == LAC_PATH_AUTO && c->B >= c->wave_decode_min_streams);
    const int vw = c->pmf_bits == 32 ? 4 : 2;
    const bool vec = (p % 16 == 0) && c->V % vw == 0 && step_stride % vw == 0 && stream_stride % vw == 0;
    const bool blockable = vec && (c->V / vw + 63) / 64 <= 512;        // per-iteration totals fit LDS
    if (blockable && (c->dpath == LAC_PATH_BLOCK || (c->dpath == LAC_PATH_AUTO && !wave &&
                                                     ((c->B >= c->block_window_lo && c->B <= c->block_window_hi) ||
                                                      c->B >= c->block_decode_min_streams)))) {
        if (c->pmf_bits == 32)
            return decode_block_launch<uint32_t, 4>(c, (const uint32_t *)pmf, step_stride, stream_stride, steps, out, st);
        return decode_block_launch<uint64_t, 2>(c, (const uint64_t *)pmf, step_stride, stream_stride, steps, out, st);
    }
    if (c->dpath == LAC_PATH_STATS || c->dpath == LAC_PATH_BLOCK || (c->dpath == LAC_PATH_AUTO && !wave)) {
        if (c->pmf_bits == 32)
            return vec ? decode_stats_path<uint32_t, 4>(c, (const uint32_t *)pmf, step_stride, stream_stride, steps, out, st)
                       : decode_stats_path<uint32_t, 1>(c, (const uint32_t *)pmf, step_stride, stream_stride, steps, out, st);
        return vec ? decode_stats_path<uint64_t, 2>(c, (const uint64_t *)pmf, step_stride, stream_stride, steps, out, st)
                   : decode_stats_path<uint64_t, 1>(c, (const uint64_t *)pmf, step_stride, stream_stride, steps, out, st);
    }
    if (wave) {
        if (c->pmf_bits == 32)
            return vec ? decode_wave_launch<uint32_t, 4>(c, (const uint32_t *)pmf, step_stride, stream_stride, steps, out, st)
                       : decode_wave_launch<uint32_t, 1>(c, (const uint32_t *)pmf, step_stride, stream_stride, steps, out, st);
        return vec ? decode_wave_launch<uint64_t, 2>(c, (const uint64_t *)pmf, step_stride, stream_stride, steps, out, st)
                   : decode_wave_launch<uint64_t, 1>(c, (const uint64_t *)pmf, step_stride, stream_stride, steps, out, st);
    }
    for (int64_t t = 0; t < steps; t++) {
        const int64_t off = t * step_stride;
        int32_t *o = out + t * c->B;
        int rc;
        const bool few = c->B <= 256;                         // 16-wave workgroups: 8 loads/lane per chunk
        if (c->pmf_bits == 32)
            rc = vec ? (few ? decode_launch<uint32_t, 4, 8>(c, (const uint32_t *)pmf, off, stream_stride, o, st)
                            : decode_launch<uint32_t, 4, 2>(c, (const uint32_t *)pmf, off, stream_stride, o, st))
                     : decode_launch<uint32_t, 1, 8>(c, (const uint32_t *)pmf, off, stream_stride, o, st);
        else
            rc = vec ? (few ? decode_launch<uint64_t, 2, 8>(c, (const uint64_t *)pmf, off, stream_stride, o, st)
                            : decode_launch<uint64_t, 2, 4>(c, (const uint64_t *)pmf, off, stream_stride, o, st))
                     : decode_launch<uint64_t, 1, 8>(c, (const uint64_t *)pmf, off, stream_stride, o, st);
        if (rc) return rc;
    }
    return LAC_OK;
}


extern "C" {

int lac_decode_open(lac_ctx *c, const uint8_t *bits_dev, uint64_t stride_bytes, const uint64_t *nbits_dev,
                    void *stream) {
    if (!c) return fail(LAC_E_ARG, "ctx is NULL");
    HIPCHK(hipSetDevice(c->device));
    if (!bits_dev) {
        bits_dev = reinterpret_cast<const uint8_t *>(c->planeA);
        stride_bytes = c->cap_words * 8;
        nbits_dev = c->nbits;
    } else {
        if (!nbits_dev) return fail(LAC_E_ARG, "nbits_dev is NULL");
        if (stride_bytes % 8 || (uintptr_t)bits_dev % 8) return fail(LAC_E_ARG, "bit buffers must be 8-byte aligned");
    }
    c->dbits = bits_dev;
    c->dstride = stride_bytes;
    c->dnbits = nbits_dev;
    c->mode = 1;
    k_dec_init<<<(unsigned)((c->B + 255) / 256), 256, 0, S(stream)>>>(c->dec, c->B, c->prec, bits_dev, stride_bytes,
                                                                      nbits_dev);
    CHECK_LAUNCH();
    return LAC_OK;
}

static_assert(sizeof(lac_dec_state) == sizeof(DecState) && offsetof(lac_dec_state, ndet) == offsetof(DecState, ndet) &&
                  offsetof(lac_dec_state, det) == offsetof(DecState, det) &&
                  offsetof(lac_dec_state, pos) == offsetof(DecState, pos),
              "lac_dec_state mirrors DecState");

int lac_decode_get_state(lac_ctx *c, lac_dec_state *host_out, void *stream) {
    if (!c || !host_out) return fail(LAC_E_ARG, "NULL argument");
    if (c->mode != 1) return fail(LAC_E_STATE, "call lac_decode_open first");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpyAsync(host_out, c->dec, sizeof(DecState) * c->B, hipMemcpyDeviceToHost, S(stream)));
    HIPCHK(hipStreamSynchronize(S(stream)));
    return LAC_OK;
}

int lac_decode_set_state(lac_ctx *c, const lac_dec_state *host_in, void *stream) {
    if (!c || !host_in) return fail(LAC_E_ARG, "NULL argument");
    if (c->mode != 1) return fail(LAC_E_STATE, "call lac_decode_open first");
    // only register sets a decoder can reach: 0 <= l < 2^(prec+1) (A_to_bin's l stays below
    // 2*denom, SURVEY finding 9), l <= h, h - l < 2^prec, pos >= prec (the kernels check x
    // against [l, h] themselves)
    const int64_t D = (int64_t)1 << c->prec;
    for (int64_t b = 0; b < c->B; b++) {
        const lac_dec_state &q = host_in[b];
        if (q.err) continue;
        if (q.l < 0 || q.l >= 2 * D || q.h < q.l || q.h - q.l >= D || q.pos < (uint64_t)c->prec ||
            q.pos > ((uint64_t)1 << 60) || q.nsym < 0 || q.ndet < 0 || (q.det != 0 && q.det != 1))
            return fail(LAC_E_ARG, "stream %lld: decoder registers out of range", (long long)b);
    }
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpyAsync(c->dec, host_in, sizeof(DecState) * c->B, hipMemcpyHostToDevice, S(stream)));
    HIPCHK(hipStreamSynchronize(S(stream)));
    return LAC_OK;
}

int lac_decode_step(lac_ctx *c, const void *pmf_dev, int64_t stream_stride, int32_t *sym_out_dev, void *stream) {
    return lac_decode_steps(c, pmf_dev, 0, stream_stride, 1, sym_out_dev, stream);
}

int lac_decode_steps(lac_ctx *c, const void *pmf_dev, int64_t step_stride, int64_t stream_stride, int64_t steps,
                     int32_t *sym_out_dev, void *stream) {
    if (!c || !pmf_dev || !sym_out_dev) return fail(LAC_E_ARG, "NULL argument");
    if (c->mode != 1) return fail(LAC_E_STATE, "call lac_decode_open first");
    if (steps < 0 || step_stride < 0 || stream_stride < 0) return fail(LAC_E_ARG, "negative size/stride");
    if (steps == 0) return LAC_OK;
    HIPCHK(hipSetDevice(c->device));
    return decode_dispatch(c, pmf_dev, step_stride, stream_stride, steps, sym_out_dev, S(stream));
}

int lac_decode_determined(lac_ctx *c, int64_t *ndet_host, void *stream) {
    if (!c || !ndet_host) return fail(LAC_E_ARG, "NULL argument");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(S(stream)));
    std::vector<DecState> v(c->B);
    HIPCHK(hipMemcpy(v.data(), c->dec, sizeof(DecState) * c->B, hipMemcpyDeviceToHost));
    for (int64_t b = 0; b < c->B; b++) ndet_host[b] = v[b].ndet;
    return LAC_OK;
}

int lac_decode_tail_begin(lac_ctx *c, void *stream) {
    if (!c) return fail(LAC_E_ARG, "ctx is NULL");
    if (c->mode != 1) return fail(LAC_E_STATE, "call lac_decode_open first");
    HIPCHK(hipSetDevice(c->device));
    if (!c->tail) HIPCHK(hipMalloc(&c->tail, sizeof(TailState) * c->B));
    k_decode_tail_begin<<<(unsigned)((c->B + 255) / 256), 256, 0, S(stream)>>>(c->dec, c->dnbits, c->B, c->prec,
                                                                               c->tail);
    CHECK_LAUNCH();
    return LAC_OK;
}

int lac_decode_tail_step(lac_ctx *c, const void *pmf_dev, int64_t stream_stride, int mode, int64_t *sym_out_dev,
                         int32_t *code_out_dev, void *stream) {
    if (!c || !sym_out_dev || !code_out_dev) return fail(LAC_E_ARG, "NULL argument");
    if (!c->tail) return fail(LAC_E_STATE, "call lac_decode_tail_begin (or lac_decode_tail_set_state) first");
    if (mode != LAC_TAIL_DECIDE && mode != LAC_TAIL_FLUSH) return fail(LAC_E_ARG, "bad tail mode %d", mode);
    if (c->mapping == LAC_MAP_CEIL && !pmf_dev) return fail(LAC_E_ARG, "pmf_dev is NULL");
    if (stream_stride < 0) return fail(LAC_E_ARG, "negative stride");
    HIPCHK(hipSetDevice(c->device));
    const int m = mode == LAC_TAIL_DECIDE ? kTailDecide : kTailFlush;
    if (c->pmf_bits == 32)
        k_decode_tail<uint32_t><<<(unsigned)c->B, kTailThreads, 0, S(stream)>>>(
            (const uint32_t *)pmf_dev, stream_stride, c->V, c->prec, c->mapping, m, c->tail, sym_out_dev, code_out_dev);
    else
        k_decode_tail<uint64_t><<<(unsigned)c->B, kTailThreads, 0, S(stream)>>>(
            (const uint64_t *)pmf_dev, stream_stride, c->V, c->prec, c->mapping, m, c->tail, sym_out_dev, code_out_dev);
    CHECK_LAUNCH();
    return LAC_OK;
}

static_assert(sizeof(lac_tail_state) == sizeof(TailState) && offsetof(lac_tail_state, err) == offsetof(TailState, err) &&
                  offsetof(lac_tail_state, nsym) == offsetof(TailState, nsym),
              "lac_tail_state mirrors TailState");

int lac_decode_tail_get_state(lac_ctx *c, lac_tail_state *host_out, void *stream) {
    if (!c || !host_out) return fail(LAC_E_ARG, "NULL argument");
    if (!c->tail) return fail(LAC_E_STATE, "no tail state: call lac_decode_tail_begin first");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpyAsync(host_out, c->tail, sizeof(TailState) * c->B, hipMemcpyDeviceToHost, S(stream)));
    HIPCHK(hipStreamSynchronize(S(stream)));
    return LAC_OK;
}

int lac_decode_tail_set_state(lac_ctx *c, const lac_tail_state *host_in, void *stream) {
    if (!c || !host_in) return fail(LAC_E_ARG, "NULL argument");
    // registers any A_from_bin holds: l <= h, lb <= hb, all within +-2^62 (the flush
    // lets l fall below 0 and h, hb exceed 2^prec; 2^62 leaves the arithmetic room)
    const int64_t lim = (int64_t)1 << 62;
    for (int64_t b = 0; b < c->B; b++) {
        const lac_tail_state &q = host_in[b];
        if (q.err) continue;
        if (q.h < q.l || q.hb < q.lb || q.l <= -lim || q.h >= lim || q.lb <= -lim || q.hb >= lim || q.still < 0 ||
            q.nsym < 0 || (q.done != 0 && q.done != 1))
            return fail(LAC_E_ARG, "stream %lld: tail registers out of range", (long long)b);
    }
    HIPCHK(hipSetDevice(c->device));
    if (!c->tail) HIPCHK(hipMalloc(&c->tail, sizeof(TailState) * c->B));
    HIPCHK(hipMemcpyAsync(c->tail, host_in, sizeof(TailState) * c->B, hipMemcpyHostToDevice, S(stream)));
    HIPCHK(hipStreamSynchronize(S(stream)));
    return LAC_OK;
}

#if LAC_DEC_PHASES
// probe builds only (tools/dec_phase_probe.sh): the k_decode_seq phase cycle sums
// (s_memtime) and the steps they cover; reset != 0 clears them
int lac_debug_dec_phases(uint64_t *out8, int reset) {
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_dec_phase), sizeof(uint64_t) * 8));
    if (reset) {
        const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_dec_phase), z, sizeof z));
    }
    return LAC_OK;
}
#endif

}  // extern "C"
