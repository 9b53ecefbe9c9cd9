// lac_dev.h -- device code shared by liblac.so's translation units (lac_api.hip,
// lac_encode.hip, lac_decode.hip, lac_logits.hip): build-time tuning knobs, wave-wide
// helpers (DPP reductions and scans), the pmf row loads and per-row reductions, the
// fudge scan (fudged_dist, arith_code.py:83-93) and the coder step with its flush and
// carry resolution (A_to_bin, :169-246).  Everything device-side sits in an anonymous
// namespace, so each translation unit compiles only what it uses.
//
// Kernels by file:
//   lac_encode.hip  k_row_stats + k_encode (split path), k_encode_fused, k_finish,
//                   k_pack (the gather's packing), reset / rebase
//   lac_decode.hip  k_decode_wave(_fine), k_decode_block, k_dec_stats + k_decode_seq,
//                   k_decode_lean, k_decode_step, the reference-frame tail (lac_tail.h)
//   lac_logits.hip  the q1 logits path: k_q1_stats (+ _rl, _wide), k_q1_decode,
//                   k_quantize_logits
//   lac_api.hip     contexts, options, status, copies, profiling, host arithmetic
#pragma once
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "lac.h"
#include "lac_core.h"
#include "lac_q1_table.h"
#include "lac_hc.h"

using namespace lac;

#define LAC_VERSION "lac-mi355x 0.1 (gfx950)"

// Row-scan tuning (tools/tune_encode.sh builds variants): vectors in flight per
// lane, and nontemporal (read-once) vs default cache policy on the row loads.
#ifndef LAC_UNROLL
#define LAC_UNROLL 8
#endif
#ifndef LAC_LEAN
#define LAC_LEAN 1          // few-stream decode: k_decode_lean ahead of k_decode_seq (probe builds set 0)
#endif
#ifndef LAC_LEAN_HELP
#define LAC_LEAN_HELP 1     // k_decode_lean: L2-prefetching helper workgroups for <= 16 streams
#endif
#ifndef LAC_NT
#define LAC_NT 1
#endif
// Minimum waves per SIMD for the one-wave-per-stream kernels (0 = no bound).
// With 4096 streams every stream's wave is resident at 4 waves/SIMD; the
// register cap spills only a few values of the per-step tail, never the row loop.
#ifndef LAC_ENC_MINW
#define LAC_ENC_MINW 0
#endif
#ifndef LAC_DEC_MINW
#define LAC_DEC_MINW 4
#endif
// k_decode_wave_fine: 2 waves/SIMD (no spills, two balanced rounds of 2048
// stream-waves at 4096 streams) measured +2.5 % over 4 (6.54 -> 6.70 TB/s).
#ifndef LAC_DECF_MINW
#define LAC_DECF_MINW 2
#endif
#if LAC_ENC_MINW > 0
#define LAC_ENC_BOUNDS __launch_bounds__(64 * LAC_STREAM_WG, LAC_ENC_MINW)
#else
#define LAC_ENC_BOUNDS __launch_bounds__(64 * LAC_STREAM_WG)
#endif
#if LAC_DEC_MINW > 0
#define LAC_DEC_BOUNDS __launch_bounds__(256, LAC_DEC_MINW)
#else
#define LAC_DEC_BOUNDS __launch_bounds__(256)
#endif

namespace {

constexpr int kChunkSteps = 64;       // split path: steps per row-stats launch at >= 512 streams
constexpr int kWavesPerBlock = 4;     // 256-thread workgroups
// one-wave-per-stream kernels (k_encode_fused, k_decode_wave(_fine)): waves per workgroup.
// 1 or 2 (a finished wave's slot refilled without waiting for its workgroup's
// slowest wave) measured no faster: c3 / c4 / u64 encode and decode within noise,
// u64 decode 13 % slower at 2 (profiles/r02/stream_wg_rejected/)
#ifndef LAC_STREAM_WG
#define LAC_STREAM_WG 4
#endif
constexpr int kStreamWaves = LAC_STREAM_WG;

// ------------------------------------------------------------------ wave helpers
__device__ inline uint32_t lane_id() { return __lane_id(); }
// The lane index recomputed by two VALU ops where it is used: an asm result the
// compiler cannot hoist, CSE or spill (a lane index held across a long loop at the
// 128-VGPR cap was spilled, and its reload's vmcnt(0) drained the loads in flight).
__device__ inline int lane_fresh() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}
// The wave's index in its workgroup as a wave-uniform (SGPR) value: the
// compiler cannot tell threadIdx.x >> 6 is uniform, so everything derived from
// it (stream index, row pointers, coder state) would otherwise occupy VGPRs.
__device__ inline int wave_in_block() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }
__device__ inline uint64_t rfl_u64(uint64_t x) {          // a wave-uniform value into SGPRs
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(x >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
}

__device__ inline uint64_t shfl_u64(uint64_t v, int src) {
    const uint32_t lo = __shfl((int)(uint32_t)v, src), hi = __shfl((int)(uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}
__device__ inline uint64_t shfl_xor_u64(uint64_t v, int m) {
    const uint32_t lo = __shfl_xor((int)(uint32_t)v, m), hi = __shfl_xor((int)(uint32_t)(v >> 32), m);
    return ((uint64_t)hi << 32) | lo;
}
__device__ inline uint64_t shfl_up_u64(uint64_t v, int d) {
    const uint32_t lo = __shfl_up((int)(uint32_t)v, d), hi = __shfl_up((int)(uint32_t)(v >> 32), d);
    return ((uint64_t)hi << 32) | lo;
}
__device__ inline i128 shfl_i128(i128 v, int src) {
    const u128 u = (u128)v;
    return (i128)(((u128)shfl_u64((uint64_t)(u >> 64), src) << 64) | shfl_u64((uint64_t)u, src));
}
__device__ inline i128 shfl_xor_i128(i128 v, int m) {
    const u128 u = (u128)v;
    return (i128)(((u128)shfl_xor_u64((uint64_t)(u >> 64), m) << 64) | shfl_xor_u64((uint64_t)u, m));
}
__device__ inline uint64_t readlane_u64(uint64_t v, int l) {
    const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
// Wave-wide reductions and scans on DPP (data-parallel primitives: VALU operand
// swizzles, a few cycles each) instead of ds_bpermute shuffles, whose LDS-path
// latency dominated the sequential per-step kernels.  Within each 16-lane row:
// quad_perm xor-1, xor-2, row_half_mirror, row_mirror leave the row's total in
// every lane; readlane of lanes 0/16/32/48 combines the four rows (uniform
// result).  The inclusive scan is Hillis-Steele over row_shr 1/2/4/8 (bound_ctrl:
// lanes shifted in from outside the row read 0), then row_bcast15 (rows 1, 3)
// and row_bcast31 (rows 2, 3).  All callers run with the whole wave active.
template <int CTRL, int ROWS = 0xF>
__device__ inline uint32_t dpp32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xF, true);
}
template <int CTRL, int ROWS = 0xF>
__device__ inline uint64_t dpp64(uint64_t v) {
    return ((uint64_t)dpp32<CTRL, ROWS>((uint32_t)(v >> 32)) << 32) | dpp32<CTRL, ROWS>((uint32_t)v);
}
enum : int { kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppHalfMirror = 0x141, kDppMirror = 0x140, kDppShr1 = 0x111,
             kDppShr2 = 0x112, kDppShr4 = 0x114, kDppShr8 = 0x118, kDppBcast15 = 0x142, kDppBcast31 = 0x143 };

// Partner exchange across lane bit BIT inside a 16-lane row, on DPP:
// bits 0/1 by quad_perm, bits 2/3 by row_shl/row_shr (each lane reads l ^ (1 << BIT)).
template <int BIT>
__device__ inline uint32_t xor_dpp(uint32_t x) {
    if constexpr (BIT == 0) return dpp32<kDppXor1>(x);
    else if constexpr (BIT == 1) return dpp32<kDppXor2>(x);
    else {
        const uint32_t up = dpp32<0x100 + (1 << BIT)>(x);    // row_shl: lane l reads l + 2^BIT
        const uint32_t dn = dpp32<0x110 + (1 << BIT)>(x);    // row_shr: lane l reads l - 2^BIT
        return ((lane_id() >> BIT) & 1) ? dn : up;
    }
}

template <typename T, typename Op>
__device__ inline T wave_reduce(T v, Op op) {
    if constexpr (sizeof(T) == 8) {
        v = op(v, (T)dpp64<kDppXor1>((uint64_t)v));
        v = op(v, (T)dpp64<kDppXor2>((uint64_t)v));
        v = op(v, (T)dpp64<kDppHalfMirror>((uint64_t)v));
        v = op(v, (T)dpp64<kDppMirror>((uint64_t)v));
        const T r0 = (T)readlane_u64((uint64_t)v, 0), r1 = (T)readlane_u64((uint64_t)v, 16);
        const T r2 = (T)readlane_u64((uint64_t)v, 32), r3 = (T)readlane_u64((uint64_t)v, 48);
        return op(op(r0, r1), op(r2, r3));
    } else {
        v = op(v, (T)dpp32<kDppXor1>((uint32_t)v));
        v = op(v, (T)dpp32<kDppXor2>((uint32_t)v));
        v = op(v, (T)dpp32<kDppHalfMirror>((uint32_t)v));
        v = op(v, (T)dpp32<kDppMirror>((uint32_t)v));
        const T r0 = (T)__builtin_amdgcn_readlane((int)v, 0), r1 = (T)__builtin_amdgcn_readlane((int)v, 16);
        const T r2 = (T)__builtin_amdgcn_readlane((int)v, 32), r3 = (T)__builtin_amdgcn_readlane((int)v, 48);
        return op(op(r0, r1), op(r2, r3));
    }
}
__device__ inline uint64_t wave_sum_u64(uint64_t v) {
    return wave_reduce(v, [](uint64_t a, uint64_t b) { return a + b; });
}
__device__ inline uint64_t wave_min_u64(uint64_t v) {
    return wave_reduce(v, [](uint64_t a, uint64_t b) { return a < b ? a : b; });
}
__device__ inline uint64_t wave_max_u64(uint64_t v) {
    return wave_reduce(v, [](uint64_t a, uint64_t b) { return a > b ? a : b; });
}
__device__ inline uint32_t wave_min_u32(uint32_t v) {
    return wave_reduce(v, [](uint32_t a, uint32_t b) { return a < b ? a : b; });
}
__device__ inline uint64_t wave_incl_scan_u64(uint64_t v) {
    v += dpp64<kDppShr1>(v);
    v += dpp64<kDppShr2>(v);
    v += dpp64<kDppShr4>(v);
    v += dpp64<kDppShr8>(v);
    v += dpp64<kDppBcast15, 0xA>(v);
    v += dpp64<kDppBcast31, 0xC>(v);
    return v;
}
__device__ inline uint32_t wave_incl_scan_u32(uint32_t v) {
    v += dpp32<kDppShr1>(v);
    v += dpp32<kDppShr2>(v);
    v += dpp32<kDppShr4>(v);
    v += dpp32<kDppShr8>(v);
    v += dpp32<kDppBcast15, 0xA>(v);
    v += dpp32<kDppBcast31, 0xC>(v);
    return v;
}
__device__ inline i128 wave_max_i128(i128 v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) { const i128 o = shfl_xor_i128(v, m); v = o > v ? o : v; }
    return v;
}
__device__ inline u128 wave_sum_u128(u128 v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1)
        v += ((u128)shfl_xor_u64((uint64_t)(v >> 64), m) << 64) | shfl_xor_u64((uint64_t)v, m);
    return v;
}
constexpr i128 kI128Min = (i128)((u128)1 << 127);

// Inclusive max-scan of an i128 over the wave on DPP (the Hillis-Steele steps of
// wave_incl_scan_u64, with lanes outside the source range reading kI128Min
// instead of 0: bound_ctrl off, `old` = the minimum's words).
template <int CTRL, int ROWS = 0xF>
__device__ inline i128 dpp_i128_or_min(i128 v) {
    const u128 u = (u128)v;
    const uint32_t w0 = (uint32_t)u, w1 = (uint32_t)(u >> 32), w2 = (uint32_t)(u >> 64), w3 = (uint32_t)(u >> 96);
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w0, CTRL, ROWS, 0xF, false);
    const uint32_t r1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w1, CTRL, ROWS, 0xF, false);
    const uint32_t r2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w2, CTRL, ROWS, 0xF, false);
    const uint32_t r3 = (uint32_t)__builtin_amdgcn_update_dpp((int)0x80000000, (int)w3, CTRL, ROWS, 0xF, false);
    return (i128)(((u128)r3 << 96) | ((u128)r2 << 64) | ((u128)r1 << 32) | r0);
}
__device__ inline i128 i128_vmax(i128 a, i128 b) { return a > b ? a : b; }
__device__ inline i128 wave_incl_max_i128(i128 v) {
    v = i128_vmax(v, dpp_i128_or_min<0x111>(v));             // row_shr:1
    v = i128_vmax(v, dpp_i128_or_min<0x112>(v));             // row_shr:2
    v = i128_vmax(v, dpp_i128_or_min<0x114>(v));             // row_shr:4
    v = i128_vmax(v, dpp_i128_or_min<0x118>(v));             // row_shr:8
    v = i128_vmax(v, dpp_i128_or_min<0x142, 0xA>(v));        // row_bcast:15 into rows 1, 3
    v = i128_vmax(v, dpp_i128_or_min<0x143, 0xC>(v));        // row_bcast:31 into rows 2, 3
    return v;
}
__device__ inline i128 readlane_i128(i128 v, int l) {
    const u128 u = (u128)v;
    return (i128)(((u128)readlane_u64((uint64_t)(u >> 64), l) << 64) | readlane_u64((uint64_t)u, l));
}

// ------------------------------------------------------------------ row loads
template <typename E, int VEC> struct VecT;
template <> struct VecT<uint32_t, 4> { typedef uint32_t type __attribute__((ext_vector_type(4))); };
template <> struct VecT<uint64_t, 2> { typedef uint64_t type __attribute__((ext_vector_type(2))); };
template <> struct VecT<uint32_t, 1> { typedef uint32_t type; };
template <> struct VecT<uint64_t, 1> { typedef uint64_t type; };

template <typename E, int VEC>
__device__ inline typename VecT<E, VEC>::type load_vec(const E *row, int64_t vi) {
    typedef typename VecT<E, VEC>::type V;
#if LAC_NT
    return __builtin_nontemporal_load(reinterpret_cast<const V *>(row) + vi);
#else
    return reinterpret_cast<const V *>(row)[vi];
#endif
}
template <typename E, int VEC>
__device__ inline E vget(const typename VecT<E, VEC>::type &v, int j) {
    if constexpr (VEC == 1) { (void)j; return v; } else { return v[j]; }
}

// Vector vi of a row when vi < nvec, else zeros -- branch-free (a clamped load and
// a select), so a predicated tail keeps all its loads in flight.  A guarded
// `vi < nvec ? load : 0` compiles to an exec-masked branch with an
// s_waitcnt vmcnt(0) inside it: one load in flight at a time.
template <typename E, int VEC>
__device__ inline typename VecT<E, VEC>::type load_vec_or0(const E *row, int64_t vi, int64_t nvec) {
    const bool ok = vi < nvec;
    const typename VecT<E, VEC>::type x = load_vec<E, VEC>(row, ok ? vi : nvec - 1);
    return ok ? x : (typename VecT<E, VEC>::type)0;
}

// ------------------------------------------------------------------ row reduction
// One wave scans a pmf row: T = sum pmf, lo = sum_{i<s} pmf, ps = pmf[s],
// minp = smallest positive entry (CDFPredictor.minp, arith_code.py:79-82) -- the
// only per-row quantities symbol_to_range (:98-110) needs when unfudged.
// u32 rows accumulate in u64 (V < 2^32 keeps it exact); u64 rows split each entry
// into 32-bit halves so a total >= 2^64 is detected instead of wrapping.
struct RowSums {
    u128 T, lo;
    uint64_t ps, minp;
};

template <typename E, int VEC>
__device__ inline RowSums row_reduce(const E *row, int64_t V, int64_t s) {
    const int lane = (int)lane_id();
    const int64_t sc = s < 0 ? 0 : (s > V ? V : s);
    const int64_t nvec = V / VEC, sfull = sc / VEC;
    const int sr = (int)(sc - sfull * VEC);
    constexpr bool W = sizeof(E) == 8;
    uint64_t tot = 0, lo = 0, tot_h = 0, lo_h = 0, ps = 0;     // *_h: high halves (u64 rows)
    E mn = (E)~(E)0;                                          // min over (x - 1): 0 wraps to max
    constexpr int U = LAC_UNROLL;
    auto take = [&](const typename VecT<E, VEC>::type &x, int64_t v) {
        uint64_t sl = 0, sh = 0;
#pragma unroll
        for (int j = 0; j < VEC; j++) {
            const E e = vget<E, VEC>(x, j);
            if constexpr (W) { sl += (uint32_t)e; sh += (uint64_t)e >> 32; } else { sl += e; }
            const E m1 = e - 1;
            mn = m1 < mn ? m1 : mn;
        }
        tot += sl;
        tot_h += sh;
        if (v < sfull) { lo += sl; lo_h += sh; }
        if (v == sfull) {                                     // the vector holding symbol s
#pragma unroll
            for (int j = 0; j < VEC; j++) {
                const E e = vget<E, VEC>(x, j);
                if (j < sr) {
                    if constexpr (W) { lo += (uint32_t)e; lo_h += (uint64_t)e >> 32; } else { lo += e; }
                }
                if (j == sr) ps = (uint64_t)e;
            }
        }
    };
    int64_t vi = lane;
    for (; vi + 64 * (U - 1) < nvec; vi += 64 * U) {
        typename VecT<E, VEC>::type x[U];
#pragma unroll
        for (int u = 0; u < U; u++) x[u] = load_vec<E, VEC>(row, vi + 64 * u);
#pragma unroll
        for (int u = 0; u < U; u++) take(x[u], vi + 64 * u);
    }
    if (vi < nvec) {                      // one predicated tail group; zero vectors add nothing
        typename VecT<E, VEC>::type x[U];
#pragma unroll
        for (int u = 0; u < U; u++)
            x[u] = load_vec_or0<E, VEC>(row, vi + 64 * u, nvec);
#pragma unroll
        for (int u = 0; u < U; u++) take(x[u], vi + 64 * u);
    }
    RowSums r;
    tot = wave_sum_u64(tot);
    lo = wave_sum_u64(lo);
    ps = wave_sum_u64(ps);
    if constexpr (W) {
        tot_h = wave_sum_u64(tot_h);
        lo_h = wave_sum_u64(lo_h);
        r.minp = wave_min_u64(mn) + 1;
    } else {
        r.minp = (uint64_t)wave_min_u32(mn) + 1;
    }
    r.T = (u128)tot + ((u128)tot_h << 32);
    r.lo = (u128)lo + ((u128)lo_h << 32);
    r.ps = ps;
    return r;
}

// The same reduction, software-pipelined across groups and rows.  A row is
// streamed in groups of U = LAC_UNROLL vectors per lane; `buf` holds the group
// being consumed while the next one is in flight (LAC_PIPE 1: the next group's
// loads are issued before the current group is consumed, 2 x U vectors in
// registers; LAC_PIPE 0: issued right after it).  After the row's last group,
// `next` (the wave's following row, or nullptr) gets its first group issued, so
// the per-step tail -- wave reductions, the coder step -- runs with loads in
// flight instead of with the wave's memory pipe idle.  On entry `buf` must hold
// group 0 of `row` (row_group_load(buf, row, 0, nvec)).
#ifndef LAC_PIPE
#define LAC_PIPE 0
#endif
// Measured on MI355X (same box, c3): no gain for the fused encoder -- u32
// 1.214 (off) vs 1.219 ms/job, u64 2.43 (off) vs 2.50 ms with a 2-wave bound
// (3.07 ms unbounded: one wave per SIMD) -- so it is off by default; the
// decoder, whose tail holds a dependent re-read, gains (LAC_DEC_XPF).
#ifndef LAC_XPF                    // issue the next row's first group before the step's tail
#define LAC_XPF 0
#endif
template <typename E, int VEC> struct RowGroup { typename VecT<E, VEC>::type x[LAC_UNROLL]; };

template <typename E, int VEC>
__device__ inline void row_group_load(RowGroup<E, VEC> &g, const E *row, int64_t base, int64_t nvec) {
    constexpr int U = LAC_UNROLL;
    const int64_t vi = base + (int64_t)lane_id();
    if (base + 64 * U <= nvec) {                              // wave-uniform: the whole group is in the row
#pragma unroll
        for (int u = 0; u < U; u++) g.x[u] = load_vec<E, VEC>(row, vi + 64 * u);
    } else {
#pragma unroll
        for (int u = 0; u < U; u++) g.x[u] = load_vec_or0<E, VEC>(row, vi + 64 * u, nvec);
    }
}

template <typename E, int VEC>
__device__ inline RowSums row_reduce_pf(const E *row, int64_t V, int64_t s, RowGroup<E, VEC> &buf, const E *next) {
    const int lane = (int)lane_id();
    const int64_t sc = s < 0 ? 0 : (s > V ? V : s);
    const int64_t nvec = V / VEC, sfull = sc / VEC;
    const int sr = (int)(sc - sfull * VEC);
    constexpr bool W = sizeof(E) == 8;
    constexpr int U = LAC_UNROLL;
    uint64_t tot = 0, lo = 0, tot_h = 0, lo_h = 0, ps = 0;
    E mn = (E)~(E)0;
    auto take = [&](const typename VecT<E, VEC>::type &x, int64_t v) {
        uint64_t sl = 0, sh = 0;
#pragma unroll
        for (int j = 0; j < VEC; j++) {
            const E e = vget<E, VEC>(x, j);
            if constexpr (W) { sl += (uint32_t)e; sh += (uint64_t)e >> 32; } else { sl += e; }
            const E m1 = e - 1;
            mn = m1 < mn ? m1 : mn;
        }
        tot += sl;
        tot_h += sh;
        if (v < sfull) { lo += sl; lo_h += sh; }
        if (v == sfull) {
#pragma unroll
            for (int j = 0; j < VEC; j++) {
                const E e = vget<E, VEC>(x, j);
                if (j < sr) {
                    if constexpr (W) { lo += (uint32_t)e; lo_h += (uint64_t)e >> 32; } else { lo += e; }
                }
                if (j == sr) ps = (uint64_t)e;
            }
        }
    };
    const int64_t gw = 64 * U, ngrp = (nvec + gw - 1) / gw;
    for (int64_t g = 0; g < ngrp; g++) {
        const int64_t base = g * gw;
#if LAC_PIPE
        const RowGroup<E, VEC> cur = buf;
        if (g + 1 < ngrp) row_group_load<E, VEC>(buf, row, base + gw, nvec);
        else if (next) row_group_load<E, VEC>(buf, next, 0, nvec);
#pragma unroll
        for (int u = 0; u < U; u++) take(cur.x[u], base + 64 * u + lane);
#else
#pragma unroll
        for (int u = 0; u < U; u++) take(buf.x[u], base + 64 * u + lane);
        if (g + 1 < ngrp) row_group_load<E, VEC>(buf, row, base + gw, nvec);
        else if (next) row_group_load<E, VEC>(buf, next, 0, nvec);
#endif
    }
    RowSums r;
    tot = wave_sum_u64(tot);
    lo = wave_sum_u64(lo);
    ps = wave_sum_u64(ps);
    if constexpr (W) {
        tot_h = wave_sum_u64(tot_h);
        lo_h = wave_sum_u64(lo_h);
        r.minp = wave_min_u64(mn) + 1;
    } else {
        r.minp = (uint64_t)wave_min_u32(mn) + 1;
    }
    r.T = (u128)tot + ((u128)tot_h << 32);
    r.lo = (u128)lo + ((u128)lo_h << 32);
    r.ps = ps;
    return r;
}

// ------------------------------------------------------------------ fudge scan
// max_{j<n} (c_j*w - j*T) over the first n entries of a row, by one wave;
// *csum (optional) receives c_{n-1}.
template <typename E>
__device__ i128 wave_xmax_prefix(const E *row, int64_t n, uint64_t w, uint64_t T, uint64_t *csum = nullptr) {
    const int lane = (int)lane_id();
    constexpr int VEC = 4;
    i128 best = kI128Min;
    uint64_t base = 0;
    E x[VEC];
    auto ld = [&](int64_t r0) {
#pragma unroll
        for (int j = 0; j < VEC; j++) {
            const int64_t e = r0 + lane * VEC + j;
            x[j] = e < n ? row[e] : (E)0;
        }
    };
    ld(0);
    for (int64_t r0 = 0; r0 < n; r0 += 64 * VEC) {
        E cur[VEC];
#pragma unroll
        for (int j = 0; j < VEC; j++) cur[j] = x[j];
        if (r0 + 64 * VEC < n) ld(r0 + 64 * VEC);                 // prefetch the next round
        uint64_t ls = 0;
#pragma unroll
        for (int j = 0; j < VEC; j++) ls += (uint64_t)cur[j];
        const uint64_t incl = wave_incl_scan_u64(ls);
        uint64_t c = base + incl - ls;
#pragma unroll
        for (int j = 0; j < VEC; j++) {
            const int64_t e = r0 + lane * VEC + j;
            c += (uint64_t)cur[j];
            if (e < n) {
                const i128 X = fudge_x(c, e, w, T);
                best = X > best ? X : best;
            }
        }
        base += readlane_u64(incl, 63);
    }
    if (csum) *csum = base;
    return wave_max_i128(best);
}

// ------------------------------------------------------------------ coder step
// receive_symbol + decide_bit/emit_bit loop of A_to_bin (arith_code.py:169-192)
// for one stream, executed uniformly by its wave.  Returns false (st.err set)
// on a coder error.
// Two quotients floor((n*m + add) / d) with one instruction stream: lane 0 divides
// n0, the other lanes n1 (the pairs of the coder step -- a and b of
// symbol_to_range, the decoder's target and its 1-padded twin -- are
// independent, and the serial per-step chain is what bounds few-stream coding).
__device__ inline void div_pair(uint64_t n0, uint64_t n1, uint64_t m, uint64_t add, uint64_t d, double inv,
                                uint64_t *q0, uint64_t *q1) {
    const uint64_t n = lane_id() == 0 ? n0 : n1;
    const uint64_t q = div_floor_inv((u128)n * m + add, d, inv);
    *q0 = readlane_u64(q, 0);
    *q1 = readlane_u64(q, 1);
}

// The same pair through precomputed row fractions (lac_core.h frac_mul_div):
// three 64-bit multiplies and one correction instead of two quotient estimates.
__device__ inline void frac_pair(uint64_t f0, uint64_t f1, uint64_t c0, uint64_t c1, uint64_t w, uint64_t T,
                                 bool ceil, uint64_t *q0, uint64_t *q1) {
    const bool first = lane_id() == 0;
    const uint64_t q = frac_mul_div(first ? f0 : f1, first ? c0 : c1, w, T, ceil);
    *q0 = readlane_u64(q, 0);
    *q1 = readlane_u64(q, 1);
}

// UNI: every argument and register is wave-uniform (k_encode keeps them in SGPRs),
// so the chain runs on the scalar unit -- the two quotients one after the other
// (a 64 x 64 -> 128-bit product is ~8 s_mul on the SALU, against four quarter-rate
// v_mad_u64_u32 plus readlanes per lane-split pair) and the fudge test as one
// compare against the row's precomputed threshold fthr = ceil(T / minp) (T > w minp
// iff w < ceil(T / minp)).
// Per-phase cycle accounting of the sequential coder steps for probe builds
// (-DLAC_ENC_PHASES=1 / -DLAC_DEC_PHASES=1, tools/enc_phase_probe.py and
// tools/dec_phase_probe.py): s_memtime deltas between marks.  The product build passes
// NoClock, whose marks compile to nothing.
struct NoClock {
    __device__ void start() {}
    __device__ void mark(int) {}
};
struct PhaseClock {
    uint64_t prev = 0, acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    __device__ void start() { prev = __builtin_amdgcn_s_memtime(); }
    __device__ void mark(int k) {
        const uint64_t now = __builtin_amdgcn_s_memtime();
        acc[k] += now - prev;
        prev = now;
    }
};
#ifndef LAC_ENC_PHASES
#define LAC_ENC_PHASES 0
#endif

// Phases marked on `clk` (probe builds): 1 the range (fudge test, two mul-divs), 2 the
// narrowing and renormalisation, 3 the plane append.
template <typename E, bool UNI = false, typename Clock = NoClock>
__device__ inline bool coder_step(EncState &st, int64_t &l, int64_t &h, uint64_t lo, uint64_t hi, uint64_t T,
                                  uint64_t minp, int64_t s, const E *row, int64_t V, int prec, uint64_t *pa,
                                  uint64_t *pc, uint64_t cap_words, uint64_t *trace_slot, int lane, int mapping,
                                  double inv_T = 0.0, bool allow_fudge = true, uint64_t flo = kNoFrac,
                                  uint64_t fhi = kNoFrac, uint64_t fthr = 0, Clock *clk = nullptr) {
    // UNI (k_encode, symbols from int32, vocab <= 2^31, w <= 2^61, fthr clamped to 2^62 by
    // the caller): 32-bit symbol test, and the fudge and zero-width tests as the signs of
    // differences -- scalar tests of a high word where a 64-bit ordered compare is a VALU
    // v_cmp plus an SGPR round trip on the chain
    if (UNI ? (uint32_t)s >= (uint32_t)V : (s < 0 || s >= V)) {   // arith_code.py:100-101
        st.err = LAC_E_SYMBOL_RANGE;
        return false;
    }
    if (T == 0) { st.err = LAC_E_TABLE; return false; }
    const uint64_t w = (uint64_t)(h - l + 1);
    uint64_t a, bb;
    if (mapping == LAC_MAP_FLOOR ||
        !(UNI ? !nonneg_uni((int64_t)(w - fthr)) : is_fudged(T, w, minp))) {   // floor: Predictor/ACSampler; else ceil
        if (UNI && flo != kNoFrac) {
            a = frac_mul_div<UNI>(flo, lo, w, T, mapping != LAC_MAP_FLOOR);
            bb = frac_mul_div<UNI>(fhi, hi, w, T, mapping != LAC_MAP_FLOOR);
        } else {
            if (flo != kNoFrac)
                frac_pair(flo, fhi, lo, hi, w, T, mapping != LAC_MAP_FLOOR, &a, &bb);
            else
                div_pair(lo, hi, w, mapping == LAC_MAP_FLOOR ? 0 : T - 1, T, inv_T != 0.0 ? inv_T : recip(T), &a,
                         &bb);
            if (UNI) {
                a = rfl_u64(a);
                bb = rfl_u64(bb);
            }
        }
    } else {                                                  // CDFPredictor.fudged_dist
        if (!allow_fudge) { st.err = LAC_E_TABLE; return false; }
        const i128 xprev = s > 0 ? wave_xmax_prefix<E>(row, s, w, T) : kI128Min;
        const i128 xs = fudge_x(hi, s, w, T);
        a = s > 0 ? fudge_f(s - 1, xprev, T, w, V) : 0;
        bb = fudge_f(s, xs > xprev ? xs : xprev, T, w, V);
        // (UNI: the wave reductions leave them in VGPRs -- uniform again here, in the
        // branches that make them, so the scalar branch's results never visit the vector
        // unit at the join, and l and h -- the chain -- stay scalar)
        if (UNI) {
            a = rfl_u64(a);
            bb = rfl_u64(bb);
        }
    }
    if (clk) clk->mark(1);
    if (UNI ? nonneg_uni((int64_t)(a - bb)) : a >= bb) { st.err = LAC_E_ZERO_WIDTH; return false; }   // the reference hangs here
    h = l + (int64_t)bb - 1;
    l = l + (int64_t)a;
    int k;
    uint64_t Ev;
    renorm(l, h, prec, &k, &Ev);
    if (clk) clk->mark(2);
    if (trace_slot && lane == 0) { trace_slot[0] = Ev; trace_slot[1] = (uint64_t)k; }
    auto store = [&](uint64_t idx, uint64_t wa, uint64_t wc) {
        if (lane == 0) { pa[idx] = wa; pc[idx] = wc; }
    };
    if (!plane_append(st.L, st.wa, st.wc, k, Ev, cap_words, store)) { st.err = LAC_E_CAPACITY; return false; }
    st.nsym++;
    if (clk) clk->mark(3);
    return true;
}

__device__ inline void store_state(EncState &st, int64_t l, int64_t h, uint64_t *pa, uint64_t *pc,
                                   uint64_t cap_words, EncState *slot) {
    if (st.err) st.err_step = st.nsym;
    if (st.L > 0 && ((st.L - 1) >> 6) < cap_words) { pa[(st.L - 1) >> 6] = st.wa; pc[(st.L - 1) >> 6] = st.wc; }
    st.l = l;
    st.h = h;
    *slot = st;
}

__host__ __device__ inline EncState fresh_state(int prec) {
    EncState st;
    memset(&st, 0, sizeof(st));
    st.l = 0;
    st.h = ((int64_t)1 << prec) - 1;
    st.nflush = -1;
    st.err_step = -1;
    return st;
}

// flush (arith_code.py:193-202) + R = A + C + F by a backward big-integer add +
// big-endian bytes (bits() :227-246, group_bits :336-347), in place.  One lane.
__device__ inline void finish_stream(EncState &st, uint64_t *pa, uint64_t *pc, uint64_t cap_words, int prec,
                                     uint64_t *nbits_slot, int term) {
    if (st.err || st.nflush >= 0) {
        *nbits_slot = st.err ? 0 : st.L;
        return;
    }
    int8_t fd[8];
    int m = 0;
    if (term == LAC_TERM_ACSAMPLER) {
        // ACSampler.flush_compress (arithmetic_coding.py:50-56): Region.step(1, 2, 3)
        // then the CarryBuffer drains -- one more floor-mapped narrowing, no digits.
        const int64_t span = st.h - st.l + 1;
        int64_t l2 = st.l + span / 3, h2 = st.l + (2 * span) / 3 - 1;
        int k;
        uint64_t Ev;
        renorm(l2, h2, prec, &k, &Ev);
        auto store = [&](uint64_t idx, uint64_t wa, uint64_t wc) { pa[idx] = wa; pc[idx] = wc; };
        if (!plane_append(st.L, st.wa, st.wc, k, Ev, cap_words, store)) {
            st.err = LAC_E_CAPACITY; st.err_step = st.nsym; *nbits_slot = 0; return;
        }
        if (st.L > 0) { pa[(st.L - 1) >> 6] = st.wa; pc[(st.L - 1) >> 6] = st.wc; }
    } else {
        m = flush_digits(st.l, st.h, prec, fd);
        if (m < 0) { st.err = LAC_E_CAPACITY; st.err_step = st.nsym; *nbits_slot = 0; return; }
    }
    int64_t F = 0;
    for (int i = 0; i < m; i++) F = F * 2 + fd[i];
    const uint64_t L = st.L, Lf = L + (uint64_t)m;
    const uint64_t nwords = (Lf + 63) >> 6;
    if (nwords > cap_words) { st.err = LAC_E_CAPACITY; st.err_step = st.nsym; *nbits_slot = 0; return; }
    const int pad = (int)(nwords * 64 - Lf);
    i128 carry = (i128)F * ((i128)1 << pad);
    const int64_t last = L ? (int64_t)((L - 1) >> 6) : -1;
    for (int64_t i = (int64_t)nwords - 1; i >= 0; i--) {
        const uint64_t a = i <= last ? pa[i] : 0, c = i <= last ? pc[i] : 0;
        const i128 sm = (i128)(u128)a + (i128)(u128)c + carry;
        pa[i] = bswap64((uint64_t)sm);
        carry = sm >> 64;
    }
    if (carry != 0) st.err = LAC_E_ARG;                   // R >= 2^L: impossible for the reference
    st.nflush = m;
    for (int i = 0; i < 8; i++) st.flush[i] = i < m ? fd[i] : 0;
    st.L = Lf;
    *nbits_slot = st.err ? 0 : Lf;
}

enum { kReset = 1, kFinish = 2 };   // encode_dispatch / q1_encode flags: job = reset + encode + finish

}  // namespace
