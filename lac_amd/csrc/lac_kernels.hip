// lac_kernels.hip -- gfx950 kernels and the C-ABI (include/lac.h) of liblac.so.
//
// Encode of one lac_encode call is two kernels per chunk of <= 64 steps:
//
//   k_row_stats   one wave per (step, stream) row.  HBM-bound scan of the integer
//                 pmf row (16-B coalesced loads, 8 in flight per lane) producing the
//                 four scalars the reference's symbol_to_range needs
//                 (arith_code.py:79-110): lo = c_{s-1}, hi = c_s, T = c_{V-1}, minp.
//   k_encode      one wave per stream, sequential over the chunk's steps: the
//                 range narrowing + renormalisation of A_to_bin (:169-192).  Lane i
//                 prefetches step i's stats; rows that hit fudged_dist (:83-93) are
//                 re-scanned by the whole wave (prefix max of c_j*w - j*T).
//
// lac_encode_finish runs k_finish (flush :193-202, carry resolution of bits()
// :227-246, MSB-first byte packing of group_bits :336-347), one lane per stream.
//
// At >= 2048 streams both directions are one launch per job with one wave per
// stream (k_encode_fused, k_decode_wave_fine); fewer streams take the split
// encode above and the block / stats decode paths.
//
// Decode (A_from_bin, :248-334): per step the row is streamed into totals, the
// search finds the chunk holding floor((x-l)*T/w), only that chunk is re-read
// and scanned to the symbol (val_to_symbol's bisect_right, :94-97), and the
// value window advances by the renormalisation (emit_bit, :284-291).
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
template <typename E, bool UNI = false>
__device__ inline bool coder_step(EncState &st, int64_t &l, int64_t &h, uint64_t lo, uint64_t hi, uint64_t T,
                                  uint64_t minp, int64_t s, const E *row, int64_t V, int prec, uint64_t *pa,
                                  uint64_t *pc, uint64_t cap_words, uint64_t *trace_slot, int lane, int mapping,
                                  double inv_T = 0.0, bool allow_fudge = true, uint64_t flo = kNoFrac,
                                  uint64_t fhi = kNoFrac, uint64_t fthr = 0) {
    if (s < 0 || s >= V) { st.err = LAC_E_SYMBOL_RANGE; return false; }   // arith_code.py:100-101
    if (T == 0) { st.err = LAC_E_TABLE; return false; }
    const uint64_t w = (uint64_t)(h - l + 1);
    uint64_t a, bb;
    if (mapping == LAC_MAP_FLOOR || !(UNI ? w < fthr : is_fudged(T, w, minp))) {  // floor: Predictor/ACSampler; else ceil
        if (UNI && flo != kNoFrac) {
            a = frac_mul_div(flo, lo, w, T, mapping != LAC_MAP_FLOOR);
            bb = frac_mul_div(fhi, hi, w, T, mapping != LAC_MAP_FLOOR);
        } else if (flo != kNoFrac)
            frac_pair(flo, fhi, lo, hi, w, T, mapping != LAC_MAP_FLOOR, &a, &bb);
        else
            div_pair(lo, hi, w, mapping == LAC_MAP_FLOOR ? 0 : T - 1, T, inv_T != 0.0 ? inv_T : recip(T), &a, &bb);
    } else {                                                  // CDFPredictor.fudged_dist
        if (!allow_fudge) { st.err = LAC_E_TABLE; return false; }
        const i128 xprev = s > 0 ? wave_xmax_prefix<E>(row, s, w, T) : kI128Min;
        const i128 xs = fudge_x(hi, s, w, T);
        a = s > 0 ? fudge_f(s - 1, xprev, T, w, V) : 0;
        bb = fudge_f(s, xs > xprev ? xs : xprev, T, w, V);
    }
    if (UNI) {                      // (the fudged branch's wave reductions leave them in VGPRs:
        a = rfl_u64(a);             //  uniform again here, or l and h -- and the chain -- would
        bb = rfl_u64(bb);           //  move to the vector unit)
    }
    if (a >= bb) { st.err = LAC_E_ZERO_WIDTH; return false; }   // the reference hangs here
    h = l + (int64_t)bb - 1;
    l = l + (int64_t)a;
    int k;
    uint64_t Ev;
    renorm(l, h, prec, &k, &Ev);
    if (trace_slot && lane == 0) { trace_slot[0] = Ev; trace_slot[1] = (uint64_t)k; }
    auto store = [&](uint64_t idx, uint64_t wa, uint64_t wc) {
        if (lane == 0) { pa[idx] = wa; pc[idx] = wc; }
    };
    if (!plane_append(st.L, st.wa, st.wc, k, Ev, cap_words, store)) { st.err = LAC_E_CAPACITY; return false; }
    st.nsym++;
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

// ------------------------------------------------------------------ split path
// k_row_stats: one wave per (step, stream) row -> RowStats.  Fully parallel over
// steps x streams: the path for small stream counts.
template <typename E, int VEC>
__global__ __launch_bounds__(256) void k_row_stats(const E *__restrict__ pmf, int64_t step_stride,
                                                   int64_t stream_stride, const int32_t *__restrict__ sym,
                                                   int64_t B, int64_t rows, int64_t V, int64_t t0,
                                                   RowStats *__restrict__ out) {
    const int lane = (int)lane_id();
    const int64_t r = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (r >= rows) return;
    const int64_t t = t0 + r / B, b = r % B;
    const RowSums rs = row_reduce<E, VEC>(pmf + t * step_stride + b * stream_stride, V, sym[t * B + b]);
    if (lane == 0) {
        RowStats st;
        if (rs.T >> 64) {
            st.lo = st.hi = st.tot = 0;
            st.minp = 1;                                  // total >= 2^64
        } else {
            st.lo = (uint64_t)rs.lo;
            st.hi = (uint64_t)rs.lo + rs.ps;
            st.tot = (uint64_t)rs.T;
            st.minp = rs.T ? rs.minp : 0;
        }
        st.inv_tot = st.tot ? 1.0 / (double)st.tot : 0.0;
        st.pad = 0;
        out[r] = st;
    }
}

// k_encode: one wave per stream over a chunk of steps; lane i prefetches the
// RowStats of step g0 + i, 64 steps at a time.
template <typename E>
__global__ __launch_bounds__(256) void k_encode(const RowStats *__restrict__ stats, const int32_t *__restrict__ sym,
                                                int64_t B, int64_t t0, int64_t nsteps, const E *pmf,
                                                int64_t step_stride, int64_t stream_stride, int64_t V, int prec,
                                                EncState *states, uint64_t *planeA, uint64_t *planeC,
                                                uint64_t cap_words, uint64_t *trace, int mapping,
                                                bool allow_fudge) {
    const int lane = (int)lane_id();
    const int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (b >= B) return;
    EncState st = states[b];
    if (st.err || st.nflush >= 0) {
        if (lane == 0 && !st.err && st.nflush >= 0) { st.err = LAC_E_STATE; st.err_step = st.nsym; states[b] = st; }
        return;
    }
    uint64_t *pa = planeA + (uint64_t)b * cap_words, *pc = planeC + (uint64_t)b * cap_words;
    // the registers and plane words wave-uniform (SGPRs): the serial chain then runs on
    // the scalar unit (coder_step<E, true>)
    int64_t l = (int64_t)rfl_u64((uint64_t)st.l), h = (int64_t)rfl_u64((uint64_t)st.h);
    st.L = rfl_u64(st.L);
    st.wa = rfl_u64(st.wa);
    st.wc = rfl_u64(st.wc);
    st.nsym = (int64_t)rfl_u64((uint64_t)st.nsym);
    bool ok = true;
    for (int64_t g0 = 0; g0 < nsteps && ok; g0 += 64) {
        const int n = (int)((nsteps - g0) < 64 ? (nsteps - g0) : 64);
        RowStats my = {0, 0, 0, 0, 0.0, 0};
        int32_t mys = 0;
        if (lane < n) {
            my = stats[(g0 + lane) * B + b];
            mys = sym[(t0 + g0 + lane) * B + b];
        }
        // the 64 steps' row fractions and fudge thresholds at once, one lane each: off
        // the serial chain
        const uint64_t flo = lane < n ? row_frac(my.lo, my.tot) : kNoFrac;
        const uint64_t fhi = lane < n ? row_frac(my.hi, my.tot) : kNoFrac;
        const uint64_t fthr = lane < n && my.minp ? div_floor((u128)my.tot + (my.minp - 1), my.minp) : 0;
        for (int i = 0; i < n; i++) {
            const uint64_t lo = readlane_u64(my.lo, i), hi = readlane_u64(my.hi, i);
            const uint64_t T = readlane_u64(my.tot, i), minp = readlane_u64(my.minp, i);
            const uint64_t invb = readlane_u64(__builtin_bit_cast(uint64_t, my.inv_tot), i);
            const uint64_t fl = readlane_u64(flo, i), fh = readlane_u64(fhi, i), ft = readlane_u64(fthr, i);
            const int64_t s = __builtin_amdgcn_readlane(mys, i);
            const int64_t t = t0 + g0 + i;
            const E *row = pmf + t * step_stride + b * stream_stride;
            if (!coder_step<E, true>(st, l, h, lo, hi, T, minp, s, row, V, prec, pa, pc, cap_words,
                                     trace ? trace + 2 * (t * B + b) : nullptr, lane, mapping,
                                     __builtin_bit_cast(double, invb), allow_fudge, fl, fh, ft)) {
                ok = false;
                break;
            }
        }
    }
    if (lane == 0) store_state(st, l, h, pa, pc, cap_words, &states[b]);
}

// ------------------------------------------------------------------ fused path
// k_encode_fused: one wave owns one stream for the whole call.  Per step it scans
// the row (HBM-bound) and applies the range update in registers, so no per-row
// statistics round-trip through HBM and no second launch; with kReset/kFinish
// the stream is also initialised and flushed + packed in the same launch.  With
// >= 2048 streams there are >= 8 waves per CU streaming rows, which hides each
// wave's short serial coder step behind the others' loads.
enum { kReset = 1, kFinish = 2 };

template <typename E, int VEC>
__global__ LAC_ENC_BOUNDS void k_encode_fused(const E *__restrict__ pmf, int64_t step_stride,
                                                      int64_t stream_stride, const int32_t *__restrict__ sym,
                                                      int64_t B, int64_t t0, int64_t nsteps, int64_t V, int prec,
                                                      EncState *states, uint64_t *planeA, uint64_t *planeC,
                                                      uint64_t cap_words, uint64_t *trace, uint64_t *nbits, int flags,
                                                      int mapping, int term) {
    const int lane = (int)lane_id();
    const int64_t b = (int64_t)blockIdx.x * kStreamWaves + (threadIdx.x >> 6);
    if (b >= B) return;
    EncState st = (flags & kReset) ? fresh_state(prec) : states[b];
    uint64_t *pa = planeA + (uint64_t)b * cap_words, *pc = planeC + (uint64_t)b * cap_words;
    if (st.err || st.nflush >= 0) {
        if (!st.err && st.nflush >= 0 && nsteps > 0) { st.err = LAC_E_STATE; st.err_step = st.nsym; }
        if (lane == 0) {
            states[b] = st;
            if (flags & kFinish) nbits[b] = st.err ? 0 : st.L;
        }
        return;
    }
    int64_t l = st.l, h = st.h;
    RowGroup<E, VEC> buf;
    if (LAC_XPF && nsteps > 0) row_group_load<E, VEC>(buf, pmf + t0 * step_stride + b * stream_stride, 0, V / VEC);
    for (int64_t i = 0; i < nsteps; i++) {
        const int64_t t = t0 + i;
        const E *row = pmf + t * step_stride + b * stream_stride;
#if LAC_XPF
        const E *next = i + 1 < nsteps ? row + step_stride : nullptr;
#else
        const E *next = nullptr;
        row_group_load<E, VEC>(buf, row, 0, V / VEC);
#endif
        const int64_t s = sym[t * B + b];
        const RowSums rs = row_reduce_pf<E, VEC>(row, V, s, buf, next);
        if (rs.T >> 64) { st.err = LAC_E_TABLE; break; }
        const uint64_t lo = (uint64_t)rs.lo;
        if (!coder_step<E>(st, l, h, lo, lo + rs.ps, (uint64_t)rs.T, rs.minp, s, row, V, prec, pa, pc, cap_words,
                           trace ? trace + 2 * (t * B + b) : nullptr, lane, mapping))
            break;
    }
    if (lane == 0) {
        store_state(st, l, h, pa, pc, cap_words, &st);
        if (flags & kFinish) finish_stream(st, pa, pc, cap_words, prec, &nbits[b], term);
        states[b] = st;
    }
}

// ------------------------------------------------------------------ k_finish
__global__ __launch_bounds__(256) void k_finish(EncState *states, uint64_t *planeA, uint64_t *planeC,
                                                uint64_t cap_words, int64_t B, int prec, uint64_t *nbits, int term) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    EncState st = states[b];
    finish_stream(st, planeA + (uint64_t)b * cap_words, planeC + (uint64_t)b * cap_words, cap_words, prec, &nbits[b],
                  term);
    states[b] = st;
}

// Drop every completed plane word of each stream, keeping the registers and the
// word that holds bit L-1 (the only bit a later carry can land on): L becomes
// ((L-1) mod 64) + 1.  For callers that take each symbol's digits from the
// trace (A_to_bin.step / run in lac_amd/coder.py) so a stream of any length
// fits a fixed capacity; the packed output of lac_encode_finish then holds
// only the tail, but the flush digits are exact.
// lac_pack_jobs / lac_pack_bits(_at): one launch packs `jobs` finished jobs back to back
// (job j's plane A at planeA + j * pstride words, its bit counts at nbits + j * B).
// Workgroup (x, j) holds streams [1024 x, 1024 x + 1024) of job j, one per thread.  Each
// workgroup first sums the byte counts ceil(nbits / 8) of everything before its own
// streams -- the earlier jobs (plus their headers) and its job's earlier streams --
// striding over them with its 1024 threads (L2-hot; a DPP wave scan and 16 wave sums
// per workgroup), then scans its own, so no workgroup waits on another.  Each thread
// writes its stream's header entry (bit count, `hdr` bytes little endian) and copies
// its packed bytes (plane A holds big-endian bytes after k_finish) behind its job's
// header, everything placed from byte `base` of dst (*base_in, 0 when NULL).
// ends[j] = the end of job j and lens[j] (when not NULL: device or host-mapped memory)
// its packed length.  A job that would pass dst_bytes writes nothing: ends[j] = its
// start, lens[j] = ~0.  (Round 4 packed one job with a one-workgroup scan launch and a
// copy launch: 7 + 4 us plus a dispatch gap, on the encode's stream, per job.)
__device__ inline uint64_t block_excl_sum1024(uint64_t v, uint64_t *wsum, uint64_t &total) {
    const int w = threadIdx.x >> 6;
    const uint64_t inc = wave_incl_scan_u64(v);
    if ((threadIdx.x & 63) == 63) wsum[w] = inc;
    __syncthreads();
    uint64_t before = 0;
    total = 0;
    for (int i = 0; i < 16; i++) {
        const uint64_t x = wsum[i];
        before += i < w ? x : 0;
        total += x;
    }
    __syncthreads();
    return before + inc - v;
}

__global__ __launch_bounds__(1024) void k_pack(const uint64_t *__restrict__ planes, uint64_t pstride,
                                               uint64_t cap_words, const uint64_t *__restrict__ nbits_all,
                                               int64_t B, int hdr, uint8_t *__restrict__ dst, uint64_t dst_bytes,
                                               const uint64_t *__restrict__ base_in, uint64_t *__restrict__ ends,
                                               uint64_t *__restrict__ lens) {
    __shared__ uint64_t wsum[16];
    const int t = threadIdx.x;
    const int64_t job = blockIdx.y, first = (int64_t)blockIdx.x * 1024, b = first + t;
    const uint64_t *nbits = nbits_all + job * B;
    const uint64_t *planeA = planes + job * pstride;
    // this thread's stream first: its count and first 4 words are in flight while the
    // workgroup sums the byte counts (plane A was written by the encode's waves on any
    // XCD, so these are L2 misses)
    const uint64_t nb = b < B ? nbits[b] : 0, n = (nb + 7) >> 3, nw = (n + 7) >> 3;
    const uint64_t *src = planeA + (uint64_t)(b < B ? b : 0) * cap_words;
    uint64_t w4[4];
#pragma unroll
    for (int i = 0; i < 4; i++) w4[i] = (uint64_t)i < nw ? src[i] : 0;
    const uint64_t base0 = base_in ? *base_in : 0;
    // bytes of the earlier jobs' streams, of this job's streams before this workgroup's,
    // and of all this job's streams (the fit test)
    uint64_t pj = 0, pw = 0, all = 0;
    for (int64_t k = t; k < (job + 1) * B; k += 1024) {
        const uint64_t m = (nbits_all[k] + 7) >> 3;
        const int64_t kj = k / B, kb = k - kj * B;
        pj += kj < job ? m : 0;
        pw += kj == job && kb < first ? m : 0;
        all += kj == job ? m : 0;
    }
    uint64_t tj, tw, ta, tb;
    (void)block_excl_sum1024(pj, wsum, tj);
    (void)block_excl_sum1024(pw, wsum, tw);
    (void)block_excl_sum1024(all, wsum, ta);
    const uint64_t excl = block_excl_sum1024(n, wsum, tb);
    const uint64_t hB = (uint64_t)hdr * (uint64_t)B, total = hB + ta;
    const uint64_t start = base0 + (uint64_t)job * hB + tj;      // job j: after the earlier jobs
    const uint64_t before_ws = tw;
    const bool fits = start <= dst_bytes && total <= dst_bytes - start;
    if (blockIdx.x == 0 && t == 0) {
        ends[job] = fits ? start + total : start;
        if (lens) lens[job] = fits ? total : ~0ull;
    }
    if (!fits || b >= B) return;
    uint8_t *h = dst + start + (uint64_t)b * hdr;
    for (int i = 0; i < hdr; i++) h[i] = (uint8_t)(nb >> (8 * i));
    uint8_t *d = dst + start + hB + before_ws + excl;
    for (uint64_t wi = 0; wi < nw; wi++) {
        const uint64_t v = wi >= 4 ? src[wi] : wi == 0 ? w4[0] : wi == 1 ? w4[1] : wi == 2 ? w4[2] : w4[3];
        const uint64_t m = n - wi * 8 < 8 ? n - wi * 8 : 8;
        for (uint64_t k = 0; k < m; k++) d[wi * 8 + k] = (uint8_t)(v >> (8 * k));
    }
}

__global__ void k_enc_rebase(EncState *states, int64_t B) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    EncState st = states[b];
    if (st.L > 64) st.L = ((st.L - 1) & 63) + 1;
    states[b] = st;
}

__global__ void k_enc_reset(EncState *states, int64_t B, int prec) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    states[b] = fresh_state(prec);
}

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

// Per-phase cycle accounting of the sequential decode step (tools/dec_phase_probe.sh
// builds a separate library with -DLAC_DEC_PHASES=1; the product build passes no clock
// and the marks compile to nothing).  Phases: 0 row totals + scan, 1 targets, 2 chunk
// search, 3 re-read + scan of the chunk, 4 ranges, 5 narrowing + renormalisation.
struct NoClock {
    __device__ void mark(int) {}
};
#ifndef LAC_DEC_PHASES
#define LAC_DEC_PHASES 0
#endif
#if LAC_DEC_PHASES
struct PhaseClock {
    uint64_t prev = 0, acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    __device__ void start() { prev = __builtin_amdgcn_s_memtime(); }
    __device__ void mark(int k) {
        const uint64_t now = __builtin_amdgcn_s_memtime();
        acc[k] += now - prev;
        prev = now;
    }
};
__device__ unsigned long long g_dec_phase[8];
#endif

// r < 0 for a wave-uniform int64.  (Forcing the test onto the scalar unit -- the high
// word's sign through an opaque SGPR, or through readfirstlane -- measured slower in both
// sequential decoders, c2 1.29 -> 1.43 / 1.50 us/step, profiles/r04/lean/: the vector
// compare it replaces overlaps.)
__device__ inline bool neg_u(uint64_t r) { return (int64_t)r < 0; }

// div_small_fix for wave-uniform values (|r| < 3d < 2^53).
__device__ inline uint64_t div_small_fix_u(uint64_t q, uint64_t n, uint64_t m, uint64_t add, uint64_t d) {
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
__device__ inline uint64_t div_small_u(uint64_t n, uint64_t m, uint64_t add, uint64_t d, double inv) {
    return div_small_fix_u(rfl_u64(div_small_est(n, m, add, inv)), n, m, add, d);
}
// Two of them with one divisor (the ranges ceil(lo*w/T), ceil(hi*w/T)): both estimates
// first, so the two FP64 chains overlap, then both corrections.
__device__ inline void div_small_u2(uint64_t n0, uint64_t n1, uint64_t m, uint64_t add, uint64_t d, double inv,
                                    uint64_t *q0, uint64_t *q1) {
    const uint64_t e0 = rfl_u64(div_small_est(n0, m, add, inv)), e1 = rfl_u64(div_small_est(n1, m, add, inv));
    *q0 = div_small_fix_u(e0, n0, m, add, d);
    *q1 = div_small_fix_u(e1, n1, m, add, d);
}

// Everything after the row's totals are known: val_to_symbol + symbol_to_range
// + advance.  `find_chunk(tgt, &cv0, &G, &cb)` locates the chunk holding tgt.
// UNI: the decoder state is wave-uniform (held in SGPRs by the caller), so the
// serial chain runs on the scalar unit with div_small's quotients where they are
// below 2^50 (prec <= 50, totals < 2^50): the few-stream decoders' step.
template <typename E, int VEC, typename FindChunk, bool UNI = false, typename Clock = NoClock, typename Idle = NoIdle>
__device__ inline int decode_symbol(DecState &st, const E *row, int64_t V, uint64_t T, uint64_t minp, int prec,
                                    int mapping, const uint8_t *bits, uint64_t nbits, FindChunk find_chunk,
                                    int64_t *s_out, Clock *clk = nullptr, Idle idle = Idle()) {
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
    if (st.det && det) st.ndet++;
    else st.det = 0;
    *s_out = s;
    const int rc = decode_advance<UNI>(st, a, bb, win, nbits, prec);
    mark(5);
    return rc;
}

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

// What k_decode_lean reads of a row whose total is below 2^32 (LEAN builds of k_dec_stats):
struct LeanMeta {
    uint64_t T;            // the total; 0: not for the lean step (bad row, T >= 2^32, minp 0)
    uint64_t fthr;         // ceil(T / minp): the ceil mapping's range is fudged iff w < fthr (arith_code.py:84)
    double iT;             // recip(T)
    uint64_t pad;
};

__device__ inline uint32_t wave_incl_scan_u32(uint32_t v) {
    v += dpp32<kDppShr1>(v);
    v += dpp32<kDppShr2>(v);
    v += dpp32<kDppShr4>(v);
    v += dpp32<kDppShr8>(v);
    v += dpp32<kDppBcast15, 0xA>(v);
    v += dpp32<kDppBcast31, 0xC>(v);
    return v;
}

// LEAN: also the row's vector-granular CDF for k_decode_lean -- vpre[row][v], the sum of
// the row's entries before vector v (mod 2^32) -- its chunks' bounds lchunk[row][lane]
// (exclusive | inclusive << 32) and a LeanMeta; exact where the total is below 2^32.
template <typename E, int VEC, bool LEAN = false>
__global__ __launch_bounds__(256) void k_dec_stats(const E *__restrict__ pmf, int64_t step_stride,
                                                   int64_t stream_stride, int64_t B, int64_t rows, int64_t V,
                                                   int64_t t0, uint64_t *__restrict__ chunks,
                                                   DecRowMeta *__restrict__ meta, uint32_t *__restrict__ vpre = nullptr,
                                                   uint64_t *__restrict__ lchunk = nullptr,
                                                   LeanMeta *__restrict__ lmeta = nullptr) {
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
    // butterfly, each added into the lane of its chunk (chunk = iteration / CI)
    int64_t chunk = 0, left = CI;
    uint32_t run = 0;                                          // LEAN: the row's sum so far, mod 2^32
    uint32_t *vp = LEAN ? vpre + r * nvec : nullptr;
    // LEAN: a group's vpre values are stored after the next group's loads are issued, so
    // the in-order wait for those loads never waits on these stores (B=64: 3.41 -> 3.35 us
    // per step; the pass stays ~1.5x the plain one, bound by its per-iteration scans)
    uint32_t pv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int64_t pg = -1;
    auto store_pending = [&]() {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int64_t vi = (pg * 8 + u) * 64 + lane;
            if (vi < nvec) vp[vi] = pv[u];
        }
    };
    for (int64_t g = 0; g < ngrp; g++) {
        typename VecT<E, VEC>::type x[8];
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
        if constexpr (LEAN) {
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const uint32_t in = wave_incl_scan_u32((uint32_t)s8[u]);
                pv[u] = run + in - (uint32_t)s8[u];
                run += (uint32_t)__builtin_amdgcn_readlane((int)in, 63);
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
        const uint32_t in = wave_incl_scan_u32((uint32_t)mine);
        lchunk[r * 64 + lane] = (uint64_t)(in - (uint32_t)mine) | ((uint64_t)in << 32);
        const uint64_t T = (uint64_t)acc128;
        const bool ok = !bad && T < (1ull << 32) && minp != 0;
        if (lane == 0)
            lmeta[r] = LeanMeta{ok ? T : 0, ok ? (T + minp - 1) / minp : 0, recip(ok ? T : 1), 0};
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
                                            const int64_t *__restrict__ resume = nullptr) {
    const int lane = (int)lane_id();
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
    uint64_t next = chunks[(i0 * B + b) * 64 + lane];
    DecRowMeta nmeta = meta[i0 * B + b];
#if LAC_DEC_PHASES
    PhaseClock clock, *clk = &clock;
    clock.start();
#else
    NoClock *clk = nullptr;
#endif
    for (int64_t i = i0; i < nsteps; i++) {
        dec_state_uniform(st);                                 // (the loop's phis are not seen as uniform)
        const int64_t t = t0 + i;
        const uint64_t mine = next;
        const DecRowMeta rm = nmeta;
        if (i + 1 < nsteps) {                                  // prefetch: independent of the state
            next = chunks[((i + 1) * B + b) * 64 + lane];
            nmeta = meta[(i + 1) * B + b];
        }
        int32_t *out = sym_out + t * B + b;
        if (st.err) {
            if (lane == 0) *out = -1;
            continue;
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
                                                                   mapping, mybits, mynbits, find_chunk, &s, clk);
        }
        if (err) {
            st.err = err;
            st.err_step = st.nsym;
        }
        if (lane == 0) *out = err ? -1 : (int32_t)s;
    }
    if (lane == 0) states[b] = st;
#if LAC_DEC_PHASES
    if (lane == 0) {
        for (int k = 0; k < 6; k++) atomicAdd(&g_dec_phase[k], (unsigned long long)clock.acc[k]);
        atomicAdd(&g_dec_phase[6], (unsigned long long)nsteps);
    }
#endif
}

// ---- lean few-stream decode step (stats path, prec <= 50, row totals < 2^32)
// k_decode_seq's serial step for what few-stream decodes nearly always are -- u32-scale
// rows (totals below 2^32), an unfudged range (or the floor mapping), prec <= 50 -- laid
// out for the latency of one wave, whose instructions issue in order.  Everything that
// depends on the row alone comes precomputed from k_dec_stats<..., LEAN>: the chunk
// bounds, T's reciprocal, the fudge threshold ceil(T/minp) and the vector-granular CDF
// vpre, loaded two steps ahead.  Left on the chain: a ballot over the chunk bounds,
// compared with the target floor(v*T/w) as products (ex*w <= v*T < in*w, no division),
// one round of loads (the chunk's entries and their vpre) with the target's division
// in its shadow, the iteration holding the target by its first vpre, a ballot over the
// lanes' cumulative sums -- no wave scan -- the two ranges and the renormalisation.  Symbols
// collect one per lane and leave in one store per 64 steps.
// Results are k_decode_seq's.  A step outside the case (a bad, large or fudged row, an
// inconsistent state or stream) ends this kernel for its stream before the step changes
// anything: resume[b] holds the step and k_decode_seq continues from it, raising the
// error if there is one.  One wave per workgroup: streams spread over the XCDs.
// Few-stream lean decode: the re-read of step i's chunk is one dependent load per step,
// an HBM round trip when the row is cold.  Helper waves -- workgroups of the same launch
// placed on the decoding wave's XCD (workgroups are dealt to the 8 XCDs round-robin, so
// index = stream mod 8) -- read one dword of every 128-B line of the rows (and vpre rows)
// a few steps ahead of the decoder, which then finds its chunk in that XCD's L2.  They
// only read: the values are discarded (an empty asm consumes them so the loads stay).
// They pace themselves by the decoder's progress (a relaxed agent-scope counter it sets
// every 8 steps), never the other way round: results do not depend on them, and a
// helper that sees no progress for ~10 ms gives up, so the grid always drains.
#ifndef LAC_LEAN_AHEAD
#define LAC_LEAN_AHEAD 16
#endif
#ifndef LAC_LEAN_HELPERS
#define LAC_LEAN_HELPERS 16
#endif
constexpr int kLeanAhead = LAC_LEAN_AHEAD;      // rows prefetched ahead of the decoder
constexpr int kLeanHelpers = LAC_LEAN_HELPERS;  // helper waves per stream
#ifndef LAC_LEAN_MAX_STREAMS
#define LAC_LEAN_MAX_STREAMS 64
#endif
constexpr int64_t kLeanMaxStreams = LAC_LEAN_MAX_STREAMS;   // k_decode_lean up to this many streams
constexpr int kLeanHelpMaxStreams = 16;         // above: no helpers (L2: ~2.6 MB ahead per stream)

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
__device__ void lean_helper(const E *pmf, int64_t step_stride, int64_t stream_stride, int64_t t0, int32_t n32,
                            int64_t V, const uint32_t *vpre, int32_t nv32, int64_t B, int64_t B8,
                            const int32_t *progress) {
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
        lean_touch(reinterpret_cast<const uint8_t *>(pmf + (t0 + t) * step_stride + b * stream_stride),
                   V * (int64_t)sizeof(E));
        lean_touch(reinterpret_cast<const uint8_t *>(vpre + ((int64_t)t * B + b) * nv32), (int64_t)nv32 * 4);
    }
}

template <typename E, int VEC, int CIM>
__global__ __launch_bounds__(64) void k_decode_lean(const E *__restrict__ pmf, int64_t step_stride,
                                                    int64_t stream_stride, int64_t t0, int64_t nsteps, int64_t V,
                                                    int prec, const uint32_t *__restrict__ vpre,
                                                    const uint64_t *__restrict__ lchunk,
                                                    const LeanMeta *__restrict__ lmeta, DecState *states,
                                                    const uint8_t *__restrict__ bits, uint64_t stride,
                                                    const uint64_t *__restrict__ nbits,
                                                    int32_t *sym_out, int64_t B, int mapping,
                                                    int64_t *__restrict__ resume, int32_t *progress) {
    typedef typename VecT<E, VEC>::type Vt;
    const int lane = (int)lane_id();
    const int64_t B8 = (B + 7) & ~(int64_t)7;
    if ((int64_t)blockIdx.x >= B8) {                             // a helper workgroup
        if (progress)
            lean_helper<E>(pmf, step_stride, stream_stride, t0, (int32_t)nsteps, V, vpre, (int32_t)(V / VEC), B, B8,
                           progress);
        return;
    }
    const int64_t b = blockIdx.x;
    if (b >= B) return;
    DecState st = states[b];
    dec_state_uniform(st);
    const uint8_t *mybits = bits + b * stride;
    const uint64_t mynbits = rfl_u64(nbits[b]);
    int64_t CI, nch;
    dec_chunk_layout<E, VEC>(V, &CI, &nch);
    const int32_t nv32 = (int32_t)(V / VEC);                    // (<= 16384: CI <= 4)
    const uint32_t ci64 = (uint32_t)CI * 64;
    const int32_t nch32 = (int32_t)nch;
    const bool ceil_map = mapping != LAC_MAP_FLOOR;
    const int32_t n32 = (int32_t)nsteps;                        // (<= chunk_steps)
    // row data two steps ahead: the lane's chunk bounds (per-lane pointer) and the LeanMeta
    // (by index, a scalar load); running pointers to row i and its vpre
    uint64_t cw = 0, cw1 = 0;
    LeanMeta lm{0, 0, 1.0, 0}, lm1{0, 0, 1.0, 0};
    if (n32 > 0) { cw = lchunk[b * 64 + lane]; lm = lmeta[b]; }
    if (n32 > 1) { cw1 = lchunk[(B + b) * 64 + lane]; lm1 = lmeta[B + b]; }
    const uint64_t *lcv = lchunk + (2 * B + b) * 64 + lane;
    int32_t li = (int32_t)(2 * B + b);
    const int32_t B32 = (int32_t)B;
    const E *rowp = pmf + t0 * step_stride + b * stream_stride;
    const uint32_t *prp = vpre + b * (int64_t)nv32;
    const int64_t pr_step = B * (int64_t)nv32;
    int32_t *outv = sym_out + (t0 + lane) * B + b;              // lane j: step 64k + j
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
    if (!st.err) {
        for (; i < n32; i++) {
            l = (int64_t)rfl_u64((uint64_t)l);                  // (the loop's phis are not seen as uniform)
            h = (int64_t)rfl_u64((uint64_t)h);
            x = (int64_t)rfl_u64((uint64_t)x);
            pos = rfl_u64(pos);
            const uint64_t T = rfl_u64(lm.T), fthr = rfl_u64(lm.fthr);
            const double iT = lm.iT;
            const uint64_t cwi = cw;
            cw = cw1;
            lm = lm1;
            if (i + 2 < n32) {                                  // row i+2
                cw1 = *lcv;
                lm1 = lmeta[li];
            }
            lcv += (int64_t)B32 * 64;
            li += B32;
            const E *row = rowp;
            const uint32_t *pr = prp;
            rowp += step_stride;
            prp += pr_step;
            const uint64_t w = (uint64_t)(h - l + 1), v = (uint64_t)(x - l);
            clk.mark(0);
            // the chunk holding tgt = floor(v*T/w) without the division: ex <= tgt < in
            // iff ex*w <= v*T < in*w, products below 2^83 as (bits 32.., bits 0..31)
            const uint64_t pl = (v & 0xffffffffull) * T, ph = (v >> 32) * T + (pl >> 32);
            const uint32_t plo = (uint32_t)pl;
            const uint32_t wl = (uint32_t)w, wh = (uint32_t)(w >> 32);
            auto le_p = [&](uint32_t e) {                       // e*w <= v*T (no short circuits: no branches)
                const uint64_t q0 = (uint64_t)e * wl, qh = (uint64_t)e * wh + (q0 >> 32);
                return (qh < ph) | ((qh == ph) & ((uint32_t)q0 <= plo));
            };
            const uint64_t cm = __ballot((lane < nch32) & le_p((uint32_t)cwi) & !le_p((uint32_t)(cwi >> 32)));
            // the chunk's loads first (in bounds whatever the step: refused below if it is bad),
            // then the stream window, then everything that can wait for them
            const uint32_t src = cm ? (uint32_t)(__ffsll((unsigned long long)cm) - 1) : 0u;
            const int32_t cv0 = (int32_t)(src * ci64);
            Vt xs[CIM];
            uint32_t ps[CIM];
#pragma unroll
            for (int g = 0; g < CIM; g++) {
                const int32_t vi = cv0 + g * 64 + lane, vc = vi < nv32 ? vi : nv32 - 1;
                xs[g] = reinterpret_cast<const Vt *>(row)[vc];
                ps[g] = pr[vc];
            }
            const BitWin win = bit_window(mybits, mynbits, pos);
            if (progress && (i & 7) == 0 && lane == 0)             // the helpers' pace (after the loads)
                __hip_atomic_store(progress + b, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // a step outside the lean case leaves at the end (a branch here would let the
            // compiler sink the loads below it); until then its divisions run on safe values
            const bool bad = (T == 0) | neg_u((uint64_t)(x - l)) | neg_u((uint64_t)(h - x)) |
                             (ceil_map & neg_u(w - fthr)) | (cm == 0);
            const uint64_t Ts = bad ? 1 : T, ws = bad ? 1 : w, vs = bad ? 0 : v;
            const double iw = recip(ws);
            const uint64_t tgt = div_small_u(vs, Ts, 0, ws, iw);   // < T < 2^32
            const uint32_t t32 = (uint32_t)tgt;
            clk.mark(1);
            // in the loads' shadow: the 1-padded end's target
            const uint64_t past = pos > mynbits ? pos - mynbits : 0;
            const int u = past < (uint64_t)prec ? (int)past : prec;
            const uint64_t vhi = vs + ((1ull << u) - 1);
            const bool vhi_in = neg_u(vhi - ws);                 // vhi < w
            const uint64_t thi = u == 0 ? tgt : (vhi_in ? div_small_u(vhi, Ts, 0, ws, iw) : 0);
            clk.mark(2);
            // the iteration holding the target: the last whose first vector starts at or below it
            int gs = 0;
#pragma unroll
            for (int g = 1; g < CIM; g++)
                if (cv0 + g * 64 < nv32 && (uint32_t)__builtin_amdgcn_readfirstlane((int)ps[g]) <= t32) gs = g;
            Vt xg = xs[0];
            uint32_t pg = ps[0];
#pragma unroll
            for (int g = 1; g < CIM; g++) {
                xg = gs == g ? xs[g] : xg;
                pg = gs == g ? ps[g] : pg;
            }
            const bool real = cv0 + gs * 64 + lane < nv32;
            uint32_t c[VEC];
            uint32_t acc = pg;
#pragma unroll
            for (int j = 0; j < VEC; j++) { acc += real ? (uint32_t)vget<E, VEC>(xg, j) : 0u; c[j] = acc; }
            const uint64_t m2 = __ballot(real & (c[VEC - 1] > t32));
            const int L = m2 ? __ffsll((unsigned long long)m2) - 1 : 0;
            uint32_t k = 0, lo = pg, hi = c[VEC - 1];
#pragma unroll
            for (int j = VEC - 1; j >= 0; j--) {
                const bool le = c[j] <= t32;
                k += le ? 1 : 0;
                hi = le ? hi : c[j];
            }
#pragma unroll
            for (int j = 0; j < VEC; j++) lo = c[j] <= t32 ? c[j] : lo;
            const uint64_t lo_c = (uint32_t)__builtin_amdgcn_readlane((int)lo, L);
            const uint64_t hi_c = (uint32_t)__builtin_amdgcn_readlane((int)hi, L);
            const int32_t sym = (cv0 + gs * 64 + L) * VEC + __builtin_amdgcn_readlane((int)k, L);
            clk.mark(3);
            uint64_t a, bb;
            div_small_u2(lo_c, hi_c, ws, ceil_map ? Ts - 1 : 0, Ts, bad ? 1.0 : iT, &a, &bb);
            // (l + a <= x <= l + bb - 1: v in [a, bb))
            if (bad || !m2 || neg_u(vs - a) || !neg_u(vs - bb)) break;
            clk.mark(4);
            if (firstnd < 0 && !(vhi_in && neg_u(thi - hi_c))) firstnd = i;
            // narrow + renormalise (decode_advance<true>)
            int64_t nl = l + (int64_t)a, nh = l + (int64_t)bb - 1;
            int kk;
            uint64_t Ev;
            renorm(nl, nh, prec, &kk, &Ev);
            if (kk > 0) {
                const BitWin wu{rfl_u64(win.w0), rfl_u64(win.w1)};
                x = (int64_t)((((uint64_t)x - (Ev << (prec - kk))) << kk) | window_bits(wu, mynbits, pos, kk));
                pos += (uint64_t)kk;
            }
            l = nl;
            h = nh;
            if (lane == (i & 63)) sbuf = sym;
            if ((i & 63) == 63) {
                *outv = sbuf;
                outv += (int64_t)B32 * 64;
            }
            clk.mark(5);
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
        resume[b] = t0 + i;
    }
}

// ================================================================ q1 logits path
// Tables computed in-kernel from logits (bf16 or f32) with the integer-exact q1
// quantiser (include/lac_q1_table.h, DESIGN.md "logits path"), so the pmf never
// exists in HBM.  Per step: pass 1 = row max, pass 2 = quantise + the usual
// reductions (the row is re-read while it is still resident in the 256 MB MALL).
__constant__ uint32_t c_q1_tab[LAC_Q1_TAB_SIZE] = LAC_Q1_TAB_INIT;

#ifndef LAC_Q1_NT
#define LAC_Q1_NT 1              // logits rows are read once: nontemporal loads
#endif
// the LDS-DMA loads of the register + slot shapes with the nt policy too: a DMA
// stream without it read at 76.5 % of peak, with it 86 % = the register loads'
// (tools/hbm_probe3.hip, profiles/r03/hbm_probe3.txt)
#ifndef LAC_Q1_DMA_NT
#define LAC_Q1_DMA_NT LAC_Q1_NT
#endif
#if LAC_Q1_DMA_NT
#define LAC_Q1_DMA_POLICY " nt"
#else
#define LAC_Q1_DMA_POLICY ""
#endif
#ifndef LAC_Q1_SCHED
#define LAC_Q1_SCHED 0           // scheduling fence between vectors in k_q1_stats
#endif
#ifndef LAC_Q1_DEFER_DEC
#define LAC_Q1_DEFER_DEC 0       // k_q1_stats decode form: a row's chunk stores after the next row's max
                                 // (measured: 3 VGPRs spilled, decode stats 42.1 -> 42.7 us per bf16 c3
                                 // step, profiles/r05/q1dec_pf/; off)
#endif

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ inline s16x2 as_s16x2(uint32_t w) {
    s16x2 r;
    __builtin_memcpy(&r, &w, 4);
    return r;
}
#ifndef LAC_Q1_IMAX
#define LAC_Q1_IMAX 1            // bf16 row max on packed int16 bit patterns (k_q1_stats)
#endif

template <typename LT> struct LogitN { static constexpr int N = 16 / sizeof(LT); };

template <typename LT>
__device__ inline float logit_at(const u32x4 &v, int j) {
    if constexpr (sizeof(LT) == 2) {
        const uint32_t w = v[j >> 1];
        return __uint_as_float((j & 1) ? (w & 0xFFFF0000u) : (w << 16));
    } else {
        return __uint_as_float(v[j]);
    }
}

__device__ inline u32x4 ld16(const void *row, int64_t vi, bool nt) {
    const u32x4 *p = reinterpret_cast<const u32x4 *>(row) + vi;
    return nt ? __builtin_nontemporal_load(p) : *p;
}

// q1 on the GPU (spec: include/lac_q1_table.h, oracle/lac_oracle.c).  With
// L = DMAX*STEPS (544): c = RNE(L - 32 m) once per row, y = fma(x, 32, c) per
// logit, j = sat_u32(y) capped at L, q = tabj[j] where the LDS tables hold
// max(1, TAB[L - j] >> (KMAX - k)) (j-indexed).  sat_u32 is v_cvt_u32_f32's own
// saturation (NaN, -inf and negatives -> 0, >= 2^32 -> 2^32-1), written as asm
// because a C++ cast of such values is undefined and the optimiser may use that.
constexpr int kQ1L = LAC_Q1_DMAX * LAC_Q1_STEPS;

__device__ inline uint32_t cvt_sat_u32(float y) {
    uint32_t r;
    asm("v_cvt_u32_f32 %0, %1" : "=v"(r) : "v"(y));
    return r;
}
__device__ inline float q1_c(float m) { return (float)kQ1L - (float)LAC_Q1_STEPS * m; }   // 32 m exact
__device__ inline uint32_t q1_j(float x, float c) {                          // general (capped) form
    const uint32_t j = cvt_sat_u32(fmaf(x, (float)LAC_Q1_STEPS, c));
    return j < (uint32_t)kQ1L ? j : (uint32_t)kQ1L;
}
// |m| < 2^18: |L - 32m| < 2^24 so c is within 0.5 of L - 32m and every y <= 544.5:
// the cap is provably idle and the fast path drops it.
__device__ inline bool q1_fast_row(float m) { return fabsf(m) < 0x1p18f; }   // false for inf / NaN

__device__ inline uint32_t q1_entry(int j, uint32_t xsh) {
    const uint32_t v = c_q1_tab[kQ1L - j] >> xsh;
    return v ? v : 1u;
}

// The per-launch j-indexed LDS table (all threads of the block, then a barrier).
__device__ inline void q1_load_tab(uint32_t *tab, uint32_t xsh) {
    for (int i = threadIdx.x; i < LAC_Q1_TAB_SIZE; i += blockDim.x) tab[i] = q1_entry(i, xsh);
    __syncthreads();
}
__device__ inline uint32_t q1_val(float x, float c, const uint32_t *tab) { return tab[q1_j(x, c)]; }

// Lane-private replicated table for the row-stats kernel: entry j, copy c at
// dword j*32 + c.  A wave64 ds_read_b32 is serviced as two 32-lane groups over 32
// banks (bank = dword mod 32); lane l reads copy l & 31, so every lookup of a
// group hits 32 distinct banks whatever the indices -- no bank conflicts for the
// random gather (a single shared copy measured 68 % conflict cycles).
#ifndef LAC_Q1_REP
#define LAC_Q1_REP 32            // table copies (power of two <= 32): lane l reads copy l % REP
#endif
#ifndef LAC_Q1_MINW
#define LAC_Q1_MINW 4            // k_q1_stats launch bound: waves per SIMD
#endif
constexpr int kQ1Rep = LAC_Q1_REP;
#ifndef LAC_Q1_FASTFILL
#define LAC_Q1_FASTFILL 1        // replicated-table fill: loads first, 16-B LDS writes
#endif
template <int REP = kQ1Rep>
__device__ inline void q1_load_tab_rep(uint32_t *tabr, uint32_t xsh) {
    for (int i = threadIdx.x; i < LAC_Q1_TAB_SIZE * REP; i += blockDim.x) tabr[i] = q1_entry(i / REP, xsh);
    __syncthreads();
}
// The same table, filled by a block of NTHR threads: entry i's REP copies are REP/4
// 16-B writes, and each thread issues all of its constant-table loads before its
// first write (the strided loop above ran 34 dependent load -> write rounds per
// thread for 32 copies at 512 threads, before any row load was issued).
template <int REP, int NTHR>
__device__ inline void q1_fill_tab_rep(uint32_t *tabr, uint32_t xsh) {
    if constexpr (!LAC_Q1_FASTFILL) {
        q1_load_tab_rep<REP>(tabr, xsh);
    } else {
        static_assert(REP % 4 == 0, "16-B writes of copies");
        constexpr int Q = REP / 4, ITEMS = LAC_Q1_TAB_SIZE * Q, IT = (ITEMS + NTHR - 1) / NTHR;
        uint32_t v[IT];
#pragma unroll
        for (int k = 0; k < IT; k++) {
            const int item = (int)threadIdx.x + k * NTHR;         // entry item / Q, copies 4 (item % Q) ..
            v[k] = item < ITEMS ? c_q1_tab[kQ1L - item / Q] : 0u;
        }
#pragma unroll
        for (int k = 0; k < IT; k++) {
            const int item = (int)threadIdx.x + k * NTHR;
            uint32_t e = v[k] >> xsh;
            e = e ? e : 1u;
            if (item < ITEMS) reinterpret_cast<u32x4 *>(tabr)[item] = u32x4{e, e, e, e};
        }
        __syncthreads();
    }
}

template <int REP = kQ1Rep>
__device__ inline uint32_t q1_rep_at(const uint32_t *tabr, uint32_t j, uint32_t loff) {
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(tabr) + ((j * (REP * 4)) | loff));
}

// Sum of q1 over the N logits of one 16-B vector (replicated table, loff = byte
// offset of this lane's copy).  Fast rows: two logits per v_pk_fma_f32, then the
// saturating conversion is the whole index computation.  Entries are <= 2^24, so
// a lane's sum of up to 128 entries fits 32 bits.
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <typename LT, int REP = kQ1Rep>
__device__ inline uint32_t q1_vec_sum(const u32x4 &x, float c, bool fast, const uint32_t *tabr, uint32_t loff) {
    constexpr int N = LogitN<LT>::N;
    uint32_t s = 0;
    if (fast) {
        const f32x2 k = {(float)LAC_Q1_STEPS, (float)LAC_Q1_STEPS}, cc = {c, c};
#pragma unroll
        for (int j = 0; j < N; j += 2) {
            const f32x2 v = {logit_at<LT>(x, j), logit_at<LT>(x, j + 1)};
            const f32x2 y = __builtin_elementwise_fma(v, k, cc);
            s += q1_rep_at<REP>(tabr, cvt_sat_u32(y.x), loff);
            s += q1_rep_at<REP>(tabr, cvt_sat_u32(y.y), loff);
        }
    } else {
#pragma unroll
        for (int j = 0; j < N; j++) s += q1_rep_at<REP>(tabr, q1_j(logit_at<LT>(x, j), c), loff);
    }
    return s;
}

__device__ inline float wave_max_f32(float v) {
    auto mx = [](uint32_t a, uint32_t b) { return __float_as_uint(fmaxf(__uint_as_float(a), __uint_as_float(b))); };
    return __uint_as_float(wave_reduce(__float_as_uint(v), mx));
}

// Sum of R per-lane values across the wave, R at once (R a power of two <= 64):
// a butterfly that halves the live values per step, so lane l ends up holding the
// total of index l / (64 / R) after R - 1 + log2(64 / R) exchanges (not R * 6).
template <int R>
__device__ inline uint64_t wave_multi_sum(uint64_t (&v)[R]) {
    const int lane = (int)lane_id();
    int m = 32;
#pragma unroll
    for (int live = R; live > 1; live >>= 1, m >>= 1) {
        const bool upper = lane & m;
#pragma unroll
        for (int i = 0; i < live / 2; i++) {
            const uint64_t keep = upper ? v[i + live / 2] : v[i];
            const uint64_t give = upper ? v[i] : v[i + live / 2];
            v[i] = keep + shfl_xor_u64(give, m);
        }
    }
    uint64_t r = v[0];
#pragma unroll
    for (int k = 32 / R; k >= 1; k >>= 1) r += shfl_xor_u64(r, k);
    return r;
}

template <int R, int BIT>
__device__ inline void multi_halve(uint32_t (&v)[R]) {
    if constexpr ((R >> BIT) > 1) {
        constexpr int live = R >> BIT;
        const bool upper = (lane_id() >> BIT) & 1;
#pragma unroll
        for (int i = 0; i < live / 2; i++) {
            const uint32_t keep = upper ? v[i + live / 2] : v[i];
            const uint32_t give = upper ? v[i] : v[i + live / 2];
            v[i] = keep + xor_dpp<BIT>(give);
        }
        multi_halve<R, BIT + 1>(v);
    }
}

// The two cross-row steps of a wave sum on gfx950's half-wave swaps (v_permlane16_swap /
// v_permlane32_swap: VALU, no LDS round trip) instead of two 64-bit ds_bpermute
// shuffles.  With x = y = v, swap(x, y) returns x with its odd rows (halves) taken from
// y's even ones and y with its even rows from x's odd ones, so x + y = v[l] + v[l ^ 16]
// (^ 32) in every lane.  r: a 16-lane row total (< 2^31); two rows can reach 2^32 (a
// flat q1 row at k = 24), so the sum widens to 64 bits first.
__device__ inline uint64_t cross_row_sum64(uint32_t r) {
    const auto a = __builtin_amdgcn_permlane16_swap(r, r, false, false);
    const uint64_t r2 = (uint64_t)a[0] + a[1];
    const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)r2, (uint32_t)r2, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(r2 >> 32), (uint32_t)(r2 >> 32), false, false);
    return (((uint64_t)hi[0] << 32) | lo[0]) + (((uint64_t)hi[1] << 32) | lo[1]);
}

// Sums of R per-lane u32 values (each < 2^27) across the wave, all R at once:
// halving steps over lane bits 0..log2(R)-1 and the rest of the 16-lane row in
// 32 bits on DPP (a row sums 16 values < 2^31), then the two cross-row steps in
// 64 bits.  Lane l ends with the total of index q_index<R>(l) (l < R distinct).
template <int R>
__device__ inline uint64_t wave_multi_sum32(uint32_t (&v)[R]) {
    static_assert(R >= 1 && R <= 16 && (R & (R - 1)) == 0, "R: power of two <= 16");
    multi_halve<R, 0>(v);
    uint32_t r = v[0];
    if constexpr (R < 2) r += xor_dpp<0>(r);
    if constexpr (R < 4) r += xor_dpp<1>(r);
    if constexpr (R < 8) r += xor_dpp<2>(r);
    if constexpr (R < 16) r += xor_dpp<3>(r);
    return cross_row_sum64(r);
}
// One halving step of multi_halve<R, BIT> for one pair (v[i], v[i + live/2]),
// so callers can run it as soon as both values exist.
template <int BIT>
__device__ inline uint32_t halve_pair(uint32_t lo, uint32_t hi) {
    const bool upper = (lane_id() >> BIT) & 1;
    return (upper ? hi : lo) + xor_dpp<BIT>(upper ? lo : hi);
}
// The end of wave_multi_sum32<8> once the caller has run all three halving steps
// itself (halve_pair<0/1/2>, see k_q1_stats_rl): r = its stage-2 value.
__device__ inline uint64_t wave_multi_sum32_tail8(uint32_t r) {
    r += xor_dpp<3>(r);
    return cross_row_sum64(r);
}
constexpr int kHalveOrder[8] = {0, 4, 2, 6, 1, 5, 3, 7};   // butterfly pairs complete early

template <int R>
__device__ inline int q_index(int lane) {                   // lane bit b -> index bit log2(R)-1-b
    int idx = 0;
#pragma unroll
    for (int b = 0; (1 << b) < R; b++) idx |= ((lane >> b) & 1) << (__builtin_ctz(R) - 1 - b);
    return idx;
}


// Row loads of k_q1_stats, two forms (RowSrc<BUF>):
//  BUF: a buffer load off one resource per row (wave-uniform row base in SGPRs,
//    one 32-bit offset VGPR per load instead of a 64-bit address), always issued:
//    lanes beyond the row load the row's last vector.  A predicated load
//    (`vi < nvec ? load : -inf`) compiles to an exec-masked branch, or a select
//    the compiler sinks below later loads; either way it ends in a vmcnt(0) that
//    waits for every load in flight -- it serialised the rolling prefetch behind
//    its own loads.  No select is needed: a duplicate of a row element cannot
//    change the row maximum, and the sums mask out-of-row vectors themselves
//    (take()).  Measured c3 bf16 0.710 -> 0.660 ms, f32 1.33 -> 1.25 ms.
//  !BUF: the predicated global load with the neutral -inf.  Kept for the
//    16-vector-per-thread shapes (V = 128256), which sit at the 128-VGPR cap:
//    there the buffer form's extra live offsets spill (3.35 -> 3.57 ms, bf16 c4).
// Callers pass a valid (uniform) row base for rows past the job.
__device__ inline u32x4 neg_inf16(int type_bytes) {
    const uint32_t w = type_bytes == 2 ? 0xFF80FF80u : 0xFF800000u;
    return u32x4{w, w, w, w};
}
template <bool BUF, int TB> struct RowSrc;
template <int TB> struct RowSrc<true, TB> {
    __amdgpu_buffer_rsrc_t rs;
    int nvec;
    __device__ RowSrc(const void *row, bool, int nv)
        : rs(__builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(row), 0, nv * 16, 0x00020000)), nvec(nv) {}
    __device__ u32x4 operator()(int vi) const {
        const uint32_t v = (uint32_t)(vi < nvec ? vi : nvec - 1);
        return __builtin_amdgcn_raw_buffer_load_b128(rs, v * 16u, 0, LAC_Q1_NT ? 2 : 0);   // 2 = nt (gfx950)
    }
};
template <int TB> struct RowSrc<false, TB> {
    const void *row;
    bool ok;
    int nvec;
    __device__ RowSrc(const void *r, bool v, int nv) : row(r), ok(v), nvec(nv) {}
    __device__ u32x4 operator()(int vi) const { return ok && vi < nvec ? ld16(row, vi, LAC_Q1_NT) : neg_inf16(TB); }
};

// k_q1_stats: the q1 row statistics.  Persistent blocks of 8 waves (two per CU:
// the replicated table takes 68 KB of LDS per block) walk the rows r = t*B + b;
// each row is owned by a group of RW waves (8/RW rows per block iteration).  Each
// thread holds R 16-B vectors of its row in registers (vector gt + NT*j of each
// NT*R-vector tile, NT = 64*RW), so a row of <= NT*R vectors is read from HBM
// exactly once: register max -> group max -> q1 sums from the same registers.
// With PF (rolling prefetch) the next row streams in while this one computes.  Longer
// rows (MULTI) take several tiles and re-read all but the last from the MALL.
//   encode (DEC = false): RowStats {lo, hi, T} of the row's symbol for k_encode;
//   decode (DEC = true):  the row max and 64 chunk totals (chunk c = vectors
//                         [c*64G, (c+1)*64G)) for k_q1_decode.
// None of this depends on the coder state, so every row of a chunk of steps runs
// in parallel and the sequential kernels only touch a few bytes per step.
constexpr int kQ1Waves = 8;

template <int R, typename Src>
__device__ inline void q1_load_tile(u32x4 (&x)[R], const Src &src, int base, int gt, int NT) {
#pragma unroll
    for (int j = 0; j < R; j++) x[j] = src(base + gt + NT * j);
}

template <typename LT, int RW, int R, bool DEC, bool MULTI, bool PF, int NWB>
__global__ __launch_bounds__(64 * NWB, LAC_Q1_MINW) void k_q1_stats(const LT *__restrict__ lg, int64_t step_stride,
                                                              int64_t stream_stride, const int32_t *__restrict__ sym,
                                                              int64_t B, int64_t rows, int64_t V, int64_t t0,
                                                              uint32_t xsh, int64_t G, RowStats *__restrict__ out,
                                                              uint64_t *__restrict__ chunks,
                                                              float *__restrict__ mrow, const uint64_t *gate) {
    // gate (the repair launch after a row-group launch, k_q1_stats_rl): run only if
    // that launch aborted its exchanges
    if (gate && __hip_atomic_load(gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
    constexpr int N = LogitN<LT>::N, NT = 64 * RW, NR = NWB / RW;
    constexpr bool IMAX = LAC_Q1_IMAX && sizeof(LT) == 2 && NR == 1 && !MULTI;
    constexpr bool BUF = R <= 8 && !MULTI;                    // row-load form (RowSrc)
    typedef RowSrc<BUF, sizeof(LT)> Src;
    static_assert(R * N <= 128, "lane sums must fit 32 bits");
    __shared__ uint32_t tabr[LAC_Q1_TAB_SIZE * kQ1Rep];
    __shared__ float smax[NWB];
    __shared__ int smaxi[NWB];
    __shared__ uint64_t ssum[NWB][2];
    __shared__ uint32_t sps[NR];
    __shared__ unsigned long long bins[DEC ? NR : 1][64];
    // in-row indices are 32-bit (vocab <= 2^31 entries); with one row per block
    // (RW = 8) the row pointer is provably wave-uniform (SGPR-based loads)
    const int tid = threadIdx.x, lane = tid & 63, w = BUF ? wave_in_block() : tid >> 6;   // BUF: SGPR rows
    const int g = NR == 1 ? 0 : w / RW, wg = NR == 1 ? w : w % RW;
    int gt = tid - g * NT;
    if (DEC && wg == 0) bins[g][lane] = 0;
    const int nvec = (int)(V / N);
    const int ntiles = MULTI ? (nvec + NT * R - 1) / (NT * R) : 1;
    const int64_t stride = (int64_t)gridDim.x * NR;
    auto row_of = [&](int64_t r) { return lg + (t0 + r / B) * step_stride + (r % B) * stream_stride; };
    u32x4 x[R];
    if (PF) {                                                  // first tile of the block's first row,
        const int64_t r0 = (int64_t)blockIdx.x * NR + g;      // in flight while the table fills
        q1_load_tile<R>(x, Src(r0 < rows ? row_of(r0) : lg, r0 < rows, nvec), 0, gt, NT);
    }
    // the 16-vector shapes sit at the 128-VGPR cap: the fast fill's live loads spill them
    // (bf16 V = 128256 decode stats 220 -> 283 us per step)
    if constexpr (R > 8) q1_load_tab_rep<kQ1Rep>(tabr, xsh);
    else q1_fill_tab_rep<kQ1Rep, 64 * NWB>(tabr, xsh);
    const uint32_t loff = (uint32_t)(lane & (kQ1Rep - 1)) << 2;
    // one 16-B vector of a tile, for the rolling prefetches
    auto ld_vec = [&](const Src &src, int tile, int j) { return src(tile * NT * R + gt + NT * j); };
    // decode form, deferred stores (LAC_Q1_DEFER_DEC): the group's writer wave keeps row
    // r's 64 chunk totals and maximum in registers and stores them once the next row's
    // maximum is taken.  A store counts in vmcnt like a load, so one issued at the row's
    // end sat in front of the waits for the next row's prefetched vectors: the writer
    // wave -- and at the next barrier its block -- waited for the store's completion.
    constexpr bool DEFER = DEC && LAC_Q1_DEFER_DEC;
    uint64_t pend_tot = 0;
    float pend_m = 0.f;
    int64_t pend_r = -1;
    auto flush_pending = [&]() {
        if (DEFER && pend_r >= 0) {
            chunks[pend_r * 64 + lane] = pend_tot;
            if (lane == 0) mrow[pend_r] = pend_m;
            pend_r = -1;
        }
    };
    for (int64_t rb = (int64_t)blockIdx.x * NR; rb < rows; rb += stride) {
        // gt opaque per row: the R per-vector lane offsets / indices derived from it are
        // recomputed (one add each) instead of hoisted out of the row loop, where
        // 2R loop-invariant VGPRs spilled the 16-vector shapes
        if (R > 8 && !DEC) asm volatile("" : "+v"(gt));          // (decode: measured neutral, spills more)
        const int64_t r = rb + g;
        const bool valid = r < rows;
        const Src row(valid ? row_of(r) : lg, valid, nvec);
        float mx = -INFINITY;
        if (MULTI) {
            // PF: tile k+1's vector j loads into x[j] as soon as tile k's max has used it
            for (int tile = 0; tile < ntiles; tile++) {
                if (!PF) q1_load_tile<R>(x, row, tile * NT * R, gt, NT);
#pragma unroll
                for (int j = 0; j < R; j++) {
#pragma unroll
                    for (int e = 0; e < N; e++) mx = fmaxf(mx, logit_at<LT>(x[j], e));
                    if (PF && tile + 1 < ntiles) {
                        x[j] = ld_vec(row, tile + 1, j);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
            }
        } else {
            if (!PF) q1_load_tile<R>(x, row, 0, gt, NT);   // PF: loaded during the last row
            if constexpr (!IMAX) {
#pragma unroll
                for (int j = 0; j < R; j++)
#pragma unroll
                    for (int e = 0; e < N; e++) mx = fmaxf(mx, logit_at<LT>(x[j], e));
            }
        }
        float m;
        if constexpr (IMAX) {
            // bf16 rows owned by the whole block: the maximum over the raw bit patterns
            // as int16 (one v_pk_max_i16 per two logits) is the float maximum whenever
            // the row has a positive, non-NaN maximum (sign-magnitude: positives order
            // as integers and beat every negative).  Other rows (all negative, or a
            // positive NaN) redo it exactly in floats from the same registers.
            s16x2 pm = {(short)-32768, (short)-32768};
#pragma unroll
            for (int j = 0; j < R; j++) {          // (.x/.y/.z/.w: a bit_cast of x[j][k] lost 3 of 4 words)
                pm = __builtin_elementwise_max(pm, as_s16x2(x[j].x));
                pm = __builtin_elementwise_max(pm, as_s16x2(x[j].y));
                pm = __builtin_elementwise_max(pm, as_s16x2(x[j].z));
                pm = __builtin_elementwise_max(pm, as_s16x2(x[j].w));
            }
            const int li = pm.x > pm.y ? (int)pm.x : (int)pm.y;
            const int wi = (int)wave_reduce((uint32_t)li, [](uint32_t a, uint32_t b) {
                return (uint32_t)((int)a > (int)b ? (int)a : (int)b);
            });
            if (lane == 0) smaxi[w] = wi;
            if (!DEC && gt == 0) sps[g] = 0;
            __syncthreads();
            int bi = smaxi[0];
#pragma unroll
            for (int i = 1; i < NWB; i++) bi = smaxi[i] > bi ? smaxi[i] : bi;
            if (bi >= 0 && bi <= 0x7F80) {                    // block-uniform
                m = __uint_as_float((uint32_t)bi << 16);
            } else {
#pragma unroll
                for (int j = 0; j < R; j++)
#pragma unroll
                    for (int e = 0; e < N; e++) mx = fmaxf(mx, logit_at<LT>(x[j], e));
                mx = wave_max_f32(mx);
                if (lane == 0) smax[w] = mx;
                __syncthreads();
                m = smax[0];
#pragma unroll
                for (int i = 1; i < NWB; i++) m = fmaxf(m, smax[i]);
            }
        } else {
            mx = wave_max_f32(mx);
            if (lane == 0) smax[w] = mx;
            if (!DEC && gt == 0) sps[g] = 0;
            __syncthreads();
            m = smax[g * RW];
#pragma unroll
            for (int i = 1; i < RW; i++) m = fmaxf(m, smax[g * RW + i]);
        }
        const bool fast = q1_fast_row(m);
        const float c = q1_c(m);
        flush_pending();                                       // the previous row's totals (DEFER)
        int sfull = -1, sr = 0;
        if (!DEC && valid) {
            const int64_t s = sym[(t0 + r / B) * B + r % B];
            const int sc = (int)(s < 0 ? 0 : (s > V ? V : s));
            sfull = sc / N;
            sr = sc - sfull * N;
        }
        uint32_t tot = 0, lo = 0;
        if (sizeof(LT) == 2) {
            // opaque to the optimiser: pass 2 re-unpacks the bf16 pairs instead of keeping
            // pass 1's 8*R unpacked floats live across the barrier (that spilled)
#pragma unroll
            for (int j = 0; j < R; j++) asm volatile("" : "+v"(x[j]));
        }
        for (int tile = ntiles - 1; tile >= 0; tile--) {
            if (MULTI && !PF && tile != ntiles - 1) q1_load_tile<R>(x, row, tile * NT * R, gt, NT);
            uint32_t sv[R];
            auto take = [&](int j, uint32_t sl) {
                const int vi = tile * NT * R + gt + NT * j;
                sl = vi < nvec ? sl : 0;
                if (DEC) {
                    sv[j] = sl;
                } else {
                    tot += sl;
                    lo += vi < sfull ? sl : 0;
                    if (vi == sfull) {                         // the vector holding s: split it once
                        uint32_t pl = 0, ps = 0;
#pragma unroll
                        for (int e = 0; e < N; e++) {
                            const uint32_t q = q1_rep_at(tabr, q1_j(logit_at<LT>(x[j], e), c), loff);
                            pl += e < sr ? q : 0;
                            ps += e == sr ? q : 0;
                        }
                        lo += pl;
                        sps[g] = ps;
                    }
                }
            };
            // rolling prefetch (PF): once vector j is consumed its registers load vector j of
            // the block's next row, so those loads overlap the rest of this row's work
            const int64_t rn = r + stride;
            const bool nvalid = rn < rows;
            const bool down = MULTI && tile > 0;              // uniform
            const Src rroll = down ? row : Src(nvalid ? row_of(rn) : lg, nvalid, nvec);
            const int troll = down ? tile - 1 : 0;
            auto roll = [&](int j) {
                if (PF) {                                      // tiles walk down: tile - 1, then the next row's tile 0
                    x[j] = ld_vec(rroll, troll, j);
                    __builtin_amdgcn_sched_barrier(0);         // keep the load after vector j's use
                }
            };
            // DEC with 8 vectors: wave_multi_sum32<8>'s butterfly runs as the sums appear
            // (vectors in the order 0 4 2 6 1 5 3 7, each halving step once both inputs
            // exist: <= 3 live sums instead of 8, as k_q1_stats_rl) -- with all 8 live
            // the rolling prefetch spilled at the 128-VGPR cap, so the decode form ran
            // without it (bf16 c3 decode stats 46-49 vs encode 41 us per step)
            constexpr bool STREAM = DEC && R == 8;
            auto pair_halve = [&](int k) {
                if constexpr (STREAM) {
                    if (k == 4) sv[0] = halve_pair<0>(sv[0], sv[4]);
                    if (k == 6) { sv[2] = halve_pair<0>(sv[2], sv[6]); sv[0] = halve_pair<1>(sv[0], sv[2]); }
                    if (k == 5) sv[1] = halve_pair<0>(sv[1], sv[5]);
                    if (k == 7) {
                        sv[3] = halve_pair<0>(sv[3], sv[7]);
                        sv[1] = halve_pair<1>(sv[1], sv[3]);
                        sv[0] = halve_pair<2>(sv[0], sv[1]);
                    }
                }
            };
            // (each halving step runs one vector late: its DPP reads a sum written a whole
            // vector earlier, not the instruction before -- DPP after a VALU write of its
            // source needs wait states, and roll()'s scheduling fence kept the compiler
            // from filling them)
            if (fast) {                                        // row-uniform branch, outside the vector loop
#pragma unroll
                for (int q = 0; q < R; q++) {
                    const int j = STREAM ? kHalveOrder[q] : q;
                    take(j, q1_vec_sum<LT>(x[j], c, true, tabr, loff));
                    if (q > 0) pair_halve(STREAM ? kHalveOrder[q - 1] : q - 1);
                    roll(j);
                }
            } else {
#pragma unroll
                for (int q = 0; q < R; q++) {
                    const int j = STREAM ? kHalveOrder[q] : q;
                    take(j, q1_vec_sum<LT>(x[j], c, false, tabr, loff));
                    if (q > 0) pair_halve(STREAM ? kHalveOrder[q - 1] : q - 1);
                    roll(j);
                }
            }
            pair_halve(STREAM ? kHalveOrder[R - 1] : R - 1);
            if (DEC) {
                uint64_t gsum;                                 // group total of index q_index(lane)
                if constexpr (STREAM) gsum = wave_multi_sum32_tail8(sv[0]);
                else gsum = wave_multi_sum32<R>(sv);
                if (lane < R) {
                    const int grp = tile * RW * R + wg + RW * q_index<R>(lane);
                    if (grp * 64 < nvec) atomicAdd(&bins[g][grp / (int)G], (unsigned long long)gsum);
                }
            }
        }
        if (!DEC) {
            const uint64_t t64 = wave_sum_u64(tot), l64 = wave_sum_u64(lo);
            if (lane == 0) { ssum[w][0] = t64; ssum[w][1] = l64; }
        }
        __syncthreads();
        if (DEC) {
            if (wg == 0) {
                if constexpr (DEFER) {
                    pend_tot = bins[g][lane];
                    pend_m = m;
                    pend_r = valid ? r : -1;
                } else {
                    if (valid) chunks[r * 64 + lane] = bins[g][lane];
                    if (valid && lane == 0) mrow[r] = m;
                }
                bins[g][lane] = 0;
            }
        } else if (gt == 0 && valid) {
            uint64_t T = 0, L = 0;
#pragma unroll
            for (int i = 0; i < RW; i++) { T += ssum[g * RW + i][0]; L += ssum[g * RW + i][1]; }
            RowStats st;
            st.lo = L;
            st.hi = L + sps[g];
            st.tot = T;
            st.minp = 1;                                       // q1 entries are >= 1
            st.inv_tot = 1.0 / (double)T;
            st.pad = 0;
            out[r] = st;
        }
    }
    flush_pending();
}

// k_q1_stats_rl: the q1 row statistics for rows of 8193..16384 16-B vectors (bf16
// V <= 131072 -- the Llama-3 c4 vocab 128256 -- and f32 V <= 65536), whose one
// row fills the register file of a CU.  One 16-wave block per CU; thread t holds
// vectors j*1024 + t of its row: j < 8 in registers, j >= 8 in its own LDS slots
// (slot k of wave w at [k*1024 + w*64, +64), written by global_load_lds, so
// the in-flight data of the next row needs no VGPRs).  Pass 2 rolls both halves
// to the block's next row as it consumes them -- an LDS slot right after its
// read, a register vector right after its use -- so the next row streams in
// while this one is quantised, instead of a CU alternating between loading a
// whole row and computing it (shape 9, 65 % of peak at c4 bf16).  LDS: REP table
// copies + the slots.  With all 8 slots (128 KB: rows up to 16384 vectors) only 8
// copies fit, and four lanes of a 32-lane LDS group share a copy: 57 % of the
// lookups' LDS cycles were bank conflicts (PMC, bf16 c4).  Rows of <= 16064
// vectors (bf16 V <= 128512: Llama-3's 128256) need only LASTN = 704 threads' worth
// of the last slot, which leaves room for 16 copies (two lanes per copy).
// Same outputs as k_q1_stats (RowStats, or row max + 64 chunk totals).
constexpr int kRLRep = 8;
constexpr int kRLLastTrim = 704;                 // last-slot threads of the 16-copy form
constexpr int kRLTrimMaxVec = 15 * 1024 + kRLLastTrim;   // rows it holds: 16064 vectors
typedef __attribute__((address_space(3))) void lvoid_t;

// NT < 1024: 1024 / NT rows per block, NT threads (NT / 64 waves) each, for
// shorter rows (c3: bf16 V = 32000 with NT = 256, f32 with NT = 512): each wave
// holds twice the vectors of the 8-wave register shapes, so the per-row
// reductions and barriers are spread over twice the bytes, and the CU keeps 4 (2)
// rows in registers + slots rolling instead of 2.  The max is taken per row; the
// IMAX fallback (float max, with its own barrier) is taken by the whole block if
// any of its rows needs it.
//
// GROUP (row groups): rows longer than one CU's registers + LDS hold (f32 V =
// 128256: Llama-3's vocab in f32; bf16 / f32 V = 151936 (Qwen2), 256000 (Gemma))
// split into kg segments of `split` vectors (the last one the rest), each held by
// one row slot (NT threads) of some block exactly as above.  Row slots are
// numbered per XCD -- slot q = (block / 8) * NRB + row-in-block of the blocks
// b = j * 8 + xcd (dispatch is round-robin over the 8 XCDs) -- and slot q holds
// segment q % kg of the XCD's row q / kg of the round: rpx rows per XCD per round,
// slots past rpx * kg idle (no loads).  Segments need not line up with blocks, so
// kg is free of the block count: with 4 rows of <= 4096 vectors per block a bf16
// Qwen2 row (18992 vectors) takes 5 slots at 93 % of their capacity, where whole
// blocks (kg = 2..4 of one or two rows each) held 77 % with 16 of 256 CUs idle.
// The segments meet twice per row: the row maximum (each slot posts its segment's
// maximum with its sequence number into one of two alternating words and polls
// its partners': the only wait; a slot's sequence counts its own exchanges, so a
// row that needs the float-max fallback exchanges once more without desynchronising
// the block's other rows), and the sums (each segment adds its partials -- total,
// lo, hi, or its 64 chunk partials -- into the row's zeroed outputs with relaxed
// device-scope atomics: no wait, and no fence -- a release/acquire fence here
// writes back / invalidates the whole L2 and cost ~35 us per row).  The grid never
// exceeds the CU count (one block per CU: every member is resident), and the wait
// is bounded: a partner that never posts poisons the row's total (+2^62:
// LAC_E_TABLE at the coder) instead of hanging the GPU.
// The exchange's wait costs ~6 points of peak at bf16 Qwen2 (the same kernel without
// it: 75 vs 69 %, wrong tables; profiles/r03/q1_slots/ab_nrb4).  Neither running the
// previous row's epilogue between the post and the poll (ab_late) nor per-row LDS
// barriers with odd rows started half a round late, so that other rows stream while
// one waits (ab_rowbar, ab_rbo), recovered any of it.
#ifndef LAC_Q1_GROUP_NOWAIT
#define LAC_Q1_GROUP_NOWAIT 0
#endif
constexpr uint32_t kGroupSpinMax = 1u << 17;                 // polls (s_sleep 2 + a device-scope load each): ~0.1 s,
                                                             // far beyond any wait for a resident partner

// DEC: a row's 64 chunk totals are stored after the NEXT row's maximum, not at the
// row's end, where the store's completion sat in front of the next row's vmcnt(0)
// (which must wait for this wave's LDS-DMA) and so in front of every wave's barrier
// (same-box A/B, profiles/r02/q1_defer/: decode stats 0-3 % faster, encode unchanged)
#ifndef LAC_Q1_DEFER
#define LAC_Q1_DEFER 1
#endif

__device__ inline uint64_t group_ld(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// post this row slot's 32-bit value (a row maximum; sequence number seq >= 1, one
// per exchange of this slot: a slot posts seq + 1 only after reading all its
// partners' seq, so no partner's word for seq is overwritten unread) and fold in
// the kg - 1 partners' (slots q0 .. q0 + kg - 1 of this XCD, q0 = (q / kg) * kg)
// with op; *ok = false when one never came.  Slot q = (b / 8) * NRB + g of block b
// uses word pair b * NRB + g.
// The launch's abort word (after the exchange words, zeroed with them): a block
// whose partner did not post within kGroupSpinMax polls -- not resident, e.g.
// while another kernel holds CUs -- sets it; every block then stops waiting at
// once (its rows are poisoned) and the gated tiled launch queued behind this one
// (q1_group_kernel) recomputes every row without row groups.
// Posting (group_post: one lane) and polling (group_poll: a whole wave, the row's
// first: lane k < kg polls partner slot q0 + k, so the kg - 1 words' L2 round trips
// overlap instead of queueing one after another; the lanes' values are folded with
// op, a wave reduction) are separate, so other work can run between them.
template <int NRB>
__device__ inline void group_post(uint64_t *xch, int g, uint32_t seq, uint32_t m) {
    const unsigned b = blockIdx.x;
    __hip_atomic_store(&xch[2 * (b * NRB + g) + (seq & 1)], ((uint64_t)seq << 32) | m, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
template <int NRB, typename Op>
__device__ inline uint32_t group_poll(uint64_t *xch, uint64_t *abortw, int g, int kg, uint32_t seq, uint32_t m,
                                      Op op, bool *ok) {
    const unsigned b = blockIdx.x, sl = seq & 1, xcd = b & 7, q = (b >> 3) * NRB + g, q0 = (q / kg) * kg;
    const unsigned lane = (unsigned)lane_fresh();
#if LAC_Q1_GROUP_NOWAIT                                          // timing experiment only: wrong tables
    *ok = true;
    return m;
#endif
    const unsigned pq = q0 + lane;
    uint32_t val = m;                                            // lanes without a partner hold the neutral m
    bool fine = true;
    if (lane < (unsigned)kg && pq != q && group_ld(abortw) == 0) {
        const unsigned pb = (pq / NRB) * 8 + xcd;
        const uint64_t *px = &xch[2 * (pb * NRB + pq % NRB) + sl];
        uint64_t v = group_ld(px);
        uint32_t n = 0;
        for (; (uint32_t)(v >> 32) != seq && n < kGroupSpinMax; n++) {
            __builtin_amdgcn_s_sleep(2);
            if ((n & 63) == 63 && group_ld(abortw)) break;       // another block gave up
            v = group_ld(px);
        }
        if ((uint32_t)(v >> 32) != seq) {
            fine = false;
            if (n >= kGroupSpinMax)
                __hip_atomic_store(abortw, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        val = (uint32_t)v;
    } else if (lane < (unsigned)kg && pq != q) {
        fine = false;                                            // the launch already gave up
    }
    *ok = __ballot(!fine) == 0;
    return wave_reduce(val, op);
}

// fmaxf of two segments' maxima (as bits): folded over all, = fmaxf over the whole row
__device__ inline uint32_t f32_max_bits(uint32_t a, uint32_t b) {
    return __float_as_uint(fmaxf(__uint_as_float(a), __uint_as_float(b)));
}

__device__ inline void group_add(uint64_t *p, uint64_t v) {
    (void)__hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr uint64_t kGroupPoison = 1ull << 62;                 // a failed exchange: the row's total is >= 2^62

template <typename LT, bool DEC, int REP = kRLRep, int LASTN = 1024, int NT = 1024, bool GROUP = false>
__global__ __launch_bounds__(1024, 4) void k_q1_stats_rl(const LT *__restrict__ lg, int64_t step_stride,
                                                         int64_t stream_stride, const int32_t *__restrict__ sym,
                                                         int64_t B, int64_t rows, int64_t V, int64_t t0, uint32_t xsh,
                                                         int64_t G, RowStats *__restrict__ out,
                                                         uint64_t *__restrict__ chunks, float *__restrict__ mrow,
                                                         uint64_t *__restrict__ xch, int split, int kg, int rpx) {
    constexpr int N = LogitN<LT>::N, R = 8, L = 8, NW = 16, NRB = 1024 / NT, NWR = NT / 64;
    constexpr int SL = (L - 1) * NT + LASTN;                   // slot vectors per row
    constexpr bool IMAX = LAC_Q1_IMAX && sizeof(LT) == 2;
    static_assert((R + L) * N <= 128, "lane sums must fit 32 bits");
    // (not the bf16 8-copy decode forms, which sit at the 128-VGPR cap: two more live
    // registers there add spills)
    constexpr bool DEFER = LAC_Q1_DEFER && !(sizeof(LT) == 2 && REP == kRLRep);
    static_assert(NT == 256 || NT == 512 || NT == 1024, "rows of 4, 8 or 16 waves");
    static_assert(LASTN % 64 == 0 && LASTN <= NT, "the last slot is trimmed by whole waves");
    constexpr bool TRIM = LASTN < NT;
    __shared__ uint32_t tabr[LAC_Q1_TAB_SIZE * REP];
    __shared__ u32x4 slots[NRB * SL];
    __shared__ float smax[NW];
    __shared__ int smaxi[NW];
    __shared__ uint64_t ssum[NW][2];
    __shared__ uint32_t sps[NRB];
    __shared__ unsigned long long gtot[DEC ? NRB * NWR * (R + L) : 1];   // DEC: every 64-vector group's total
    int tid = threadIdx.x;
    const int lane = tid & 63, w = wave_in_block();
    const int g = w / NWR, wg = w % NWR;                      // this wave's row of the block, wave in that row
    // (the fast fill below the first row's loads, as in k_q1_stats, spilled this
    // kernel at its 128-VGPR cap: 2.52 -> 2.70 ms at bf16 V = 128256)
    q1_load_tab_rep<REP>(tabr, xsh);
    const uint32_t loff = (uint32_t)(lane & (REP - 1)) << 2;
    // GROUP: row slot q (of this XCD) holds segment hh = q % kg of the XCD's row q / kg
    // of each round (rows r = round * 8 * rpx + (q / kg) * 8 + xcd); segments are split
    // vectors long, the last one the rest; slots past rpx * kg are idle
    const int sq = (int)(blockIdx.x >> 3) * NRB + g;
    const int hh = GROUP ? sq % kg : 0;
    const bool idle = GROUP && sq / kg >= rpx;                  // wave-uniform
    const int vofs = hh * split;                                // vectors of the row before this segment
    const int nvec = GROUP ? (idle ? 1 : hh < kg - 1 ? split : (int)(V / N) - (kg - 1) * split) : (int)(V / N);
    // TRIM: waves past LASTN have no last slot (their vectors there lie beyond the row)
    const bool noslot = TRIM && wg * 64 >= LASTN;
    // rows r = base + roff, base = b0, b0 + stride, ... < rows (the same count in every
    // block of a group launch: partners exchange once per round)
    const int64_t stride = GROUP ? 8 * (int64_t)rpx : (int64_t)gridDim.x * NRB;
    const int64_t b0 = GROUP ? 0 : (int64_t)blockIdx.x * NRB;
    const int64_t roff = GROUP ? (int64_t)(sq / kg) * 8 + (blockIdx.x & 7) : g;
    auto row_of = [&](int64_t r) {
        return lg + (t0 + r / B) * step_stride + (r % B) * stream_stride + (int64_t)vofs * N;
    };
    __shared__ uint32_t sxv[NRB];
    __shared__ int sxok[NRB];
    __shared__ int sxact[NRB];
    uint32_t seq = 0;                                           // GROUP: this row slot's exchanges
    bool pok = true;                                            // GROUP: every exchange of this row came
    // GROUP: this segment's value v for the row, posted, and then folded with the
    // partners' (block-wide calls with the same v and act; only rows with act --
    // row-uniform, and the same in every segment of a row -- exchange, the others
    // keep v)
    auto group_post_v = [&](uint32_t v, bool act) {
        seq += act ? 1 : 0;
        if (act && tid == g * NT) group_post<NRB>(xch, g, seq, v);
    };
    auto group_poll_v = [&](uint32_t v, bool act, auto op) {
        if (wg == 0) {                                          // each row's first wave (wave-uniform)
            bool ok = true;
            const uint32_t res = act ? group_poll<NRB>(xch, xch + 2 * NRB * gridDim.x, g, kg, seq, v, op, &ok) : v;
            if (tid == g * NT) {
                sxv[g] = res;
                sxok[g] = ok;
                sxact[g] = act;
            }
        }
        __syncthreads();
        pok = pok && sxok[g] != 0;
        return sxv[g];
    };
    auto group_combine = [&](uint32_t v, bool act, auto op) {
        group_post_v(v, act);
        return group_poll_v(v, act, op);
    };
    int64_t pend_r = -1;                                        // DEC, LAC_Q1_DEFER: a row's chunk totals
    uint64_t pend = 0;                                          //   (lane ln: chunk ln) not yet stored
    auto flush_chunks = [&]() {
        if (pend_r < 0) return;
        const int ln = lane_fresh();
        if constexpr (GROUP) {                                  // into the zeroed chunk totals
            if (pend) group_add(&chunks[pend_r * 64 + ln], pend);
        } else {
            chunks[pend_r * 64 + ln] = pend;
        }
        pend_r = -1;
    };
    auto gti = [&]() { return tid - g * NT; };                 // thread index in the row
    // vector j of this thread (clamped into the row: a duplicate cannot change the
    // maximum, and the sums mask out-of-row vectors)
    auto vidx = [&](int j) { const int vi = j * NT + gti(); return vi < nvec ? vi : nvec - 1; };
    auto ld_reg = [&](const RowSrc<true, sizeof(LT)> &src, int j) { return src(j * NT + gti()); };
    // LDS-DMA as asm: the compiler's own global_load_lds makes every later LDS read
    // wait vmcnt(0) (it cannot tell the slots apart), which serialised the refills.
    // The asm is invisible to its wait counting, so this kernel waits explicitly:
    // vmcnt(0) before pass 1 reads any slot, lgkmcnt(0) before a slot is refilled.
    const uint32_t slot_base = (uint32_t)(uintptr_t)(lvoid_t *)&slots[g * SL + wg * 64];   // wave-uniform
    auto ld_lds = [&](const LT *rw, int k) {
        if ((k == L - 1 && noslot) || idle) return;            // wave-uniform
        const u32x4 *src = reinterpret_cast<const u32x4 *>(rw) + vidx(R + k);
        uint32_t keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" LAC_Q1_DMA_POLICY "\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(src), "s"(slot_base + (uint32_t)(k * NT * 16))
                     : "memory");
    };
    // a row's epilogue, after the barrier that follows its pass 2: its partials (wave
    // sums, the symbol's entry, DEC: group totals) into the outputs
    auto epilogue = [&](int64_t er, bool eok) {
        if constexpr (DEC) {
            if (wg == 0 && er >= 0) {
                // chunk c = groups [c G, (c + 1) G) of the row's ngrp groups
                // GROUP: this segment's groups are the row's [gofs, gofs + ngrp) (split is a multiple of 64)
                const int ngrp = (nvec + 63) / 64, ln = lane_fresh(), gofs = vofs / 64;
                const int g0 = ln * (int)G, ga = g0 > gofs ? g0 : gofs;
                const int gb = g0 + (int)G < gofs + ngrp ? g0 + (int)G : gofs + ngrp;
                uint64_t ct = 0;
                for (int gi = ga; gi < gb; gi++) ct += gtot[g * NWR * (R + L) + gi - gofs];
                pend = ct + (GROUP && !eok ? kGroupPoison : 0);
                pend_r = er;
                if (!DEFER) flush_chunks();
            }
        } else if (gti() == 0) {
            const uint64_t ps = sps[g];
            if (er < 0) return;
            uint64_t T = 0, Ls = 0;
#pragma unroll
            for (int i = 0; i < NWR; i++) { T += ssum[g * NWR + i][0]; Ls += ssum[g * NWR + i][1]; }
            if constexpr (GROUP) {                              // the segments' partials add up
                RowStats *o = out + er;                        // (zeroed; inv_tot 0: the coder divides)
                group_add(&o->tot, T + (eok ? 0 : kGroupPoison));
                group_add(&o->lo, Ls);
                group_add(&o->hi, Ls + ps);
                if (hh == 0) __hip_atomic_store(&o->minp, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                RowStats st;
                st.lo = Ls;
                st.hi = Ls + ps;
                st.tot = T;
                st.minp = 1;
                st.inv_tot = 1.0 / (double)T;
                st.pad = 0;
                out[er] = st;
            }
        }
    };
    u32x4 x[R];
    {                                                          // the block's first rows
        const int64_t r0 = b0 + roff;
        const LT *rw = r0 < rows ? row_of(r0) : lg;
        const RowSrc<true, sizeof(LT)> src(rw, true, idle ? 0 : nvec);   // idle: no loads (out of range: 0)
#pragma unroll
        for (int k = 0; k < L; k++) ld_lds(rw, k);
#pragma unroll
        for (int j = 0; j < R; j++) x[j] = ld_reg(src, j);
    }
    for (int64_t rb = b0; rb < rows; rb += stride) {
        // tid opaque per row: the per-load addresses derived from it are recomputed
        // next to each load, not hoisted out of the loop and spilled (a spill reload
        // is a VM load: its vmcnt(0) would drain the prefetches)
        asm volatile("" : "+v"(tid));
        const int64_t r = rb + roff;
        const bool valid = !idle && r < rows;
        const int64_t rn = r + stride;
        const LT *nrow = rn < rows ? row_of(rn) : lg;
        // pass 1: the row maximum over registers and slots (everything has landed)
        __builtin_amdgcn_s_waitcnt(0);                         // this wave's LDS-DMA writes (asm: untracked)
        asm volatile("" ::: "memory");
        // slot vectors are read where used (not held across the barrier: registers)
        // (a wave without a last slot reads the neutral -inf: no other wave's DMA
        // writes are waited for here, and those vectors are masked from the sums)
        auto slot = [&](int k) {
            return (k == L - 1 && noslot) ? neg_inf16(sizeof(LT)) : slots[g * SL + k * NT + gti()];
        };
        float m;
        pok = true;
        if constexpr (IMAX) {
            s16x2 pm = {(short)-32768, (short)-32768};
            auto pmax = [&](const u32x4 &v) {
                pm = __builtin_elementwise_max(pm, as_s16x2(v.x));
                pm = __builtin_elementwise_max(pm, as_s16x2(v.y));
                pm = __builtin_elementwise_max(pm, as_s16x2(v.z));
                pm = __builtin_elementwise_max(pm, as_s16x2(v.w));
            };
#pragma unroll
            for (int j = 0; j < R; j++) pmax(x[j]);
#pragma unroll
            for (int k = 0; k < L; k++) pmax(slot(k));
            const int li = pm.x > pm.y ? (int)pm.x : (int)pm.y;
            const int wi = (int)wave_reduce((uint32_t)li, [](uint32_t a, uint32_t b) {
                return (uint32_t)((int)a > (int)b ? (int)a : (int)b);
            });
            if (lane == 0) smaxi[w] = wi;
            if (!DEC && gti() == 0) sps[g] = 0;
            __syncthreads();
            int bi = 0;
            bool all_ok = true;                                // block-uniform: every row's int max usable
#pragma unroll
            for (int gg = 0; gg < NRB; gg++) {
                int bm = smaxi[gg * NWR];
#pragma unroll
                for (int i = 1; i < NWR; i++) bm = smaxi[gg * NWR + i] > bm ? smaxi[gg * NWR + i] : bm;
                all_ok = all_ok && bm >= 0 && bm <= 0x7F80;
                bi = gg == g ? bm : bi;
            }
            bool my_ok = true;                                 // GROUP: this row's combined int max usable
            if constexpr (GROUP) {                              // one row: the int max of all segments
                bi = (int)group_combine((uint32_t)bi, valid, [](uint32_t a, uint32_t b) {
                    return (int)a > (int)b ? a : b;
                });
                my_ok = !valid || (bi >= 0 && bi <= 0x7F80);
                all_ok = true;                                 // (block-uniform: every exchanging row's combined max)
#pragma unroll
                for (int gg = 0; gg < NRB; gg++)
                    all_ok = all_ok && (!sxact[gg] || ((int)sxv[gg] >= 0 && (int)sxv[gg] <= 0x7F80));
            }
            if (all_ok) {                                      // (see k_q1_stats)
                m = __uint_as_float((uint32_t)bi << 16);
            } else {
                float mx = -INFINITY;
#pragma unroll
                for (int j = 0; j < R; j++)
#pragma unroll
                    for (int e = 0; e < N; e++) mx = fmaxf(mx, logit_at<LT>(x[j], e));
#pragma unroll
                for (int k = 0; k < L; k++) {
                    const u32x4 v = slot(k);
#pragma unroll
                    for (int e = 0; e < N; e++) mx = fmaxf(mx, logit_at<LT>(v, e));
                }
                mx = wave_max_f32(mx);
                if (lane == 0) smax[w] = mx;
                __syncthreads();
                m = smax[g * NWR];
#pragma unroll
                for (int i = 1; i < NWR; i++) m = fmaxf(m, smax[g * NWR + i]);
                if constexpr (GROUP) {                          // only the rows whose int max failed exchange again
                    const float mf = __uint_as_float(group_combine(
                        __float_as_uint(m), valid && !my_ok, [](uint32_t a, uint32_t b) { return f32_max_bits(a, b); }));
                    m = my_ok ? __uint_as_float((uint32_t)bi << 16) : mf;
                }
            }
        } else {
            float mx = -INFINITY;
#pragma unroll
            for (int j = 0; j < R; j++)
#pragma unroll
                for (int e = 0; e < N; e++) mx = fmaxf(mx, logit_at<LT>(x[j], e));
#pragma unroll
            for (int k = 0; k < L; k++) {
                const u32x4 v = slot(k);
#pragma unroll
                for (int e = 0; e < N; e++) mx = fmaxf(mx, logit_at<LT>(v, e));
            }
            mx = wave_max_f32(mx);
            if (lane == 0) smax[w] = mx;
            if (!DEC && gti() == 0) sps[g] = 0;
            __syncthreads();
            m = smax[g * NWR];
#pragma unroll
            for (int i = 1; i < NWR; i++) m = fmaxf(m, smax[g * NWR + i]);
            if constexpr (GROUP)
                m = __uint_as_float(group_combine(__float_as_uint(m), valid,
                                                  [](uint32_t a, uint32_t b) { return f32_max_bits(a, b); }));
        }
        if (DEC && valid && gti() == 0 && hh == 0) mrow[r] = m;   // now: m is not held over pass 2
        if constexpr (DEC) flush_chunks();                    // the previous row's (LAC_Q1_DEFER)
        const bool fast = q1_fast_row(m);
        const float c = q1_c(m);
        int sfull = -1, sr = 0;
        if (!DEC && valid) {
            const int64_t s = sym[(t0 + r / B) * B + r % B];
            const int sc = (int)(s < 0 ? 0 : (s > V ? V : s));
            sfull = sc / N;
            sr = sc - sfull * N;
            sfull -= vofs;                                     // GROUP: < 0 in a segment past the one holding s
        }
        uint32_t tot = 0, lo = 0, sv[8];                     // DEC: one half's vector sums
        if (!DEC && sfull >= 0 && sfull < nvec && (sfull & (NT - 1)) == gti()) {
            // the vector holding s, split once before pass 2 (both halves still hold
            // this row): one copy of this code instead of one per vector in pass 2
            const int js = sfull / NT;
            u32x4 v = js >= R ? slot(js - R) : x[0];
#pragma unroll
            for (int jj = 1; jj < R; jj++) v = js == jj ? x[jj] : v;
            uint32_t pl = 0, ps = 0;
#pragma unroll
            for (int e = 0; e < N; e++) {
                const uint32_t q = q1_rep_at<REP>(tabr, q1_j(logit_at<LT>(v, e), c), loff);
                pl += e < sr ? q : 0;
                ps += e == sr ? q : 0;
            }
            lo = pl;
            sps[g] = ps;
        }
        // pass 2 (slots first, so their refills are issued earliest)
        auto take = [&](int j, const u32x4 &v, uint32_t sl) {
            const int vi = j * NT + gti();
            sl = vi < nvec ? sl : 0;
            if (DEC) {
                sv[j & 7] = sl;
            } else {
                tot += sl;
                lo += vi < sfull ? sl : 0;
            }
            (void)v;
        };
        const RowSrc<true, sizeof(LT)> nsrc(nrow, true, idle ? 0 : nvec);
        // DEC: the 64-vector group totals of one half (vectors j0 .. j0+7) into the bins,
        // by wave_multi_sum32<8>'s butterfly run as the sums appear: vectors are taken in
        // the order 0 4 2 6 1 5 3 7 and each halving step runs once both of its inputs
        // exist, so at most 3 sums are live instead of 8 (the 8-live form spilled at the
        // 128-VGPR cap).  Same totals, lane for lane.
        auto bin_half = [&](int j0) {
            const uint64_t gsum = wave_multi_sum32_tail8(sv[0]);   // lane l < 8: index q_index<8>(l)
            // each group has one writer: a plain LDS store (no division by G, no atomics;
            // the chunk totals are summed from these after the row's barrier)
            // (lane_fresh: the lane and its bit-reversed index are recomputed here rather
            // than held across the row loop -- held, they spilled, and the reload's
            // vmcnt(0) waited for the next row's slot loads just issued)
            const int ln = lane_fresh();
            if (ln < 8) gtot[g * NWR * (R + L) + wg + NWR * (j0 + q_index<8>(ln))] = gsum;   // [grp*64, +64)
        };
        auto pair_halve = [&](int k) {                         // k: the vector just taken (compile-time)
            if (!DEC) return;
            if (k == 4) sv[0] = halve_pair<0>(sv[0], sv[4]);
            if (k == 6) { sv[2] = halve_pair<0>(sv[2], sv[6]); sv[0] = halve_pair<1>(sv[0], sv[2]); }
            if (k == 5) sv[1] = halve_pair<0>(sv[1], sv[5]);
            if (k == 7) {
                sv[3] = halve_pair<0>(sv[3], sv[7]);
                sv[1] = halve_pair<1>(sv[1], sv[3]);
                sv[0] = halve_pair<2>(sv[0], sv[1]);
            }
        };
        auto pass2 = [&](bool fs) {
#pragma unroll
            for (int q = 0; q < L; q++) {
                const int k = DEC ? kHalveOrder[q] : q;
                const u32x4 v = slot(k);
                take(R + k, v, q1_vec_sum<LT, REP>(v, c, fs, tabr, loff));
                pair_halve(k);
                __builtin_amdgcn_s_waitcnt(0xc07f);           // lgkmcnt(0): this wave's reads of slot k are done
                ld_lds(nrow, k);
                __builtin_amdgcn_sched_barrier(0);
            }
            if (DEC) bin_half(R);
#pragma unroll
            for (int q = 0; q < R; q++) {
                const int j = DEC ? kHalveOrder[q] : q;
                take(j, x[j], q1_vec_sum<LT, REP>(x[j], c, fs, tabr, loff));
                pair_halve(j);
                x[j] = ld_reg(nsrc, j);
                __builtin_amdgcn_sched_barrier(0);
            }
            if (DEC) bin_half(0);
        };
        if (fast) pass2(true); else pass2(false);             // row-uniform (a wave is in one row)
        if (!DEC) {
            const uint64_t t64 = wave_sum_u64(tot), l64 = wave_sum_u64(lo);
            if (lane == 0) { ssum[w][0] = t64; ssum[w][1] = l64; }
        }
        __syncthreads();
        epilogue(valid ? r : -1, pok);
    }
    if constexpr (DEC) flush_chunks();
    __builtin_amdgcn_s_waitcnt(0);                             // no LDS-DMA outlives the block
    asm volatile("" ::: "memory");
}

// k_q1_stats_wide (shape 22): one row per CU held entirely in registers by an
// 8-wave block at 2 waves per SIMD (256 VGPRs per lane): thread t holds vectors
// t + 512 j, j < R, of its row -- R = 40: rows of <= 20480 16-B vectors (bf16
// V <= 163840: Qwen2's 151936; f32 V <= 81920).  The 16-wave shapes hold only 8
// vectors per thread in registers (128-VGPR cap, most of it working registers),
// so such rows had to be split over row slots of several blocks with a maximum
// exchange between them (§5b item 14); with 8 waves the register file is mostly
// row, no exchange.  All R loads of a row are issued at once, so a CU alternates a
// load phase and a compute phase (~4 VALU ops per logit); the CUs drift apart, so
// the chip's HBM stream stays busy while some of them compute.  LDS: the 32-copy
// table only (no bank conflicts).  Same outputs as k_q1_stats.
//
// GROUP (shape 23): rows longer than one block holds (bf16 Gemma 256000 / 262144,
// f32 Llama-3 / Qwen2 / Gemma) in kg segments of `split` vectors (the last one the
// rest), one per block, exactly as the row slots of k_q1_stats_rl's GROUP form
// with one row per block: slot q = block / 8 of the block's XCD holds segment
// q % kg of the XCD's row q / kg of each round (rpx rows per XCD per round, grid =
// 8 rpx kg <= the CU count: every member resident), the segments exchange the row
// maximum through group_post / group_poll and add their partials into the zeroed
// outputs with relaxed atomics; a partner that never posts sets the launch's abort
// word and poisons the row, and the gated repair launch recomputes every row.
template <typename LT, int R, bool DEC, bool GROUP = false, int L = 0>
__global__ __launch_bounds__(512, 2) void k_q1_stats_wide(const LT *__restrict__ lg, int64_t step_stride,
                                                          int64_t stream_stride, const int32_t *__restrict__ sym,
                                                          int64_t B, int64_t rows, int64_t V, int64_t t0, uint32_t xsh,
                                                          int64_t G, RowStats *__restrict__ out,
                                                          uint64_t *__restrict__ chunks, float *__restrict__ mrow,
                                                          uint64_t *__restrict__ xch, int split, int kg, int rpx) {
    constexpr int N = LogitN<LT>::N, NT = 512, NW = 8;
    constexpr bool IMAX = LAC_Q1_IMAX && sizeof(LT) == 2;
    static_assert(R % 8 == 0, "group totals in batches of 8 vectors");
    __shared__ uint32_t tabr[LAC_Q1_TAB_SIZE * kQ1Rep];
    __shared__ float smax[NW];
    __shared__ int smaxi[NW];
    __shared__ uint64_t ssum[NW][2];
    __shared__ uint32_t sps;
    __shared__ unsigned long long bins[DEC ? 64 : 1];
    __shared__ uint32_t sxv;
    __shared__ int sxok;
    // L > 0: vectors j = R .. R + L - 1 of each thread in LDS slots (slot k of thread t
    // at slots[k NT + t], filled by LDS-DMA), for rows of NT R < vectors <= NT (R + L)
    __shared__ u32x4 slots[L > 0 ? L * NT : 1];
    const int tid = threadIdx.x, lane = tid & 63, w = wave_in_block();
    // GROUP: this block's segment of its rows (slot sq of its XCD)
    const int sq = (int)(blockIdx.x >> 3), hh = GROUP ? sq % kg : 0;
    const int vofs = hh * split;                               // vectors of the row before the segment
    const int nrow = (int)(V / N);
    const int nvec = GROUP ? (hh < kg - 1 ? split : nrow - (kg - 1) * split) : nrow;
    const int64_t stride = GROUP ? 8 * (int64_t)rpx : (int64_t)gridDim.x;
    const int64_t r0 = GROUP ? (int64_t)(sq / kg) * 8 + (blockIdx.x & 7) : (int64_t)blockIdx.x;
    auto row_of = [&](int64_t r) {
        return lg + (t0 + r / B) * step_stride + (r % B) * stream_stride + (int64_t)vofs * N;
    };
    // one buffer resource per row (SGPRs) sized to the row: vector tid + 512 j at
    // voffset tid * 16 + soffset j * 8192, one offset VGPR for all R loads; loads past
    // the row return 0 without touching memory, and pass 1 masks those vectors
    auto rsrc = [&](int64_t r) {                               // no row (r >= rows): 0 bytes, loads return 0
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<LT *>(r < rows ? row_of(r) : lg), 0,
                                                 r < rows ? nvec * 16 : 0, 0x00020000);
    };
    // GROUP: post this segment's value for the row and fold in the partners' (block-wide)
    uint32_t seq = 0;
    bool pok = true;                                           // every exchange of this row came
    auto group_combine = [&](uint32_t v, auto op) {
        seq++;
        if (tid == 0) group_post<1>(xch, 0, seq, v);
        if (w == 0) {
            bool ok = true;
            const uint32_t res = group_poll<1>(xch, xch + 2 * gridDim.x, 0, kg, seq, v, op, &ok);
            if (lane == 0) {
                sxv = res;
                sxok = ok;
            }
        }
        __syncthreads();
        pok = pok && sxok != 0;
        return sxv;
    };
    auto load_vec = [&](const __amdgpu_buffer_rsrc_t &rs, int j) {
        // soffset materialised next to its load (asm): 40 hoisted constants spilled SGPRs
        uint32_t so;
        asm volatile("s_mov_b32 %0, %1" : "=s"(so) : "i"(j * NT * 16));
        return __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)tid * 16u, so, LAC_Q1_NT ? 2 : 0);
    };
    // LDS-DMA as asm (see k_q1_stats_rl: untracked by the compiler's wait counting, so
    // pass 1 waits vmcnt(0) itself and a slot is refilled after lgkmcnt(0)); lanes past
    // the row load its last vector (masked when read)
    const uint32_t slot_base = (uint32_t)(uintptr_t)(lvoid_t *)&slots[w * 64];   // wave-uniform
    auto ld_slot = [&](const LT *rw, int k, int ti_, int nv_) {
        // (ti_, nv_ opaque per row: 11 hoisted clamped offsets spilled the bf16 decode form)
        const int vi = ti_ + NT * (R + k);
        const u32x4 *src = reinterpret_cast<const u32x4 *>(rw) + (vi < nv_ ? vi : nv_ - 1);
        uint32_t keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" LAC_Q1_DMA_POLICY "\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(src), "s"(slot_base + (uint32_t)(k * NT * 16))
                     : "memory");
    };
    u32x4 x[R];
    {                                                          // the first row, in flight during the table fill
        const __amdgpu_buffer_rsrc_t rs = rsrc(r0);
#pragma unroll
        for (int j = 0; j < R; j++) x[j] = load_vec(rs, j);
        if (L > 0 && r0 < rows) {
#pragma unroll
            for (int kk = 0; kk < L; kk++) ld_slot(row_of(r0), kk, tid, nvec);
        }
    }
    if (DEC && w == 0) bins[lane] = 0;
    q1_fill_tab_rep<kQ1Rep, NT>(tabr, xsh);
    const uint32_t loff = (uint32_t)(lane & (kQ1Rep - 1)) << 2;
    // the q1 weight of a -inf logit (index 0) -- what every vector past the row adds in
    // pass 2 once pass 1 has made it -inf; subtracted from the totals instead of masking
    // each vector (per-vector masks are loop-invariant: hoisted, they spilled)
    const uint32_t tab0 = q1_entry(0, xsh);
    // decode: group grp's chunk, grp / G, by a multiply with m = ceil(2^32 / G) (exact
    // for grp * G < 2^32; groups < 2^16 here): per-lane divisions by the runtime G were
    // hoisted out of the row loop, one per batch, and spilled
    const bool g1 = G <= 1;                                    // (m = 2^32 does not fit: G = 1 is the identity)
    const uint32_t gmag = g1 ? 0u : (uint32_t)((0xFFFFFFFFull + (uint64_t)G) / (uint64_t)G);
    auto chunk_of = [&](int grp) { return g1 ? grp : (int)__umulhi((uint32_t)grp, gmag); };
    for (int64_t r = r0; r < rows; r += stride) {          // (GROUP: a group's members share r)
        // (the row was loaded during the previous row's pass 2: rolling prefetch)
        pok = true;
        // tid and nvec opaque per row: what is derived from them is recomputed where it
        // is used instead of hoisted out of the row loop into live registers
        int ti = tid, nv = nvec;
        asm volatile("" : "+v"(ti), "+s"(nv));
        // vectors past the row read as 0: -inf for the maximum (vectors j >= nv / NT only)
        const int nfull = nv / NT;
#pragma unroll
        for (int j = 0; j < R; j++)
            if (j >= nfull) x[j] = ti + NT * j < nv ? x[j] : neg_inf16(sizeof(LT));
        if constexpr (L > 0) {                                 // this wave's LDS-DMA writes (asm: untracked)
            __builtin_amdgcn_s_waitcnt(0);
            asm volatile("" ::: "memory");
        }
        // slot vector k, read where used (past the row: -inf)
        auto slot = [&](int kk) {
            const u32x4 v = slots[kk * NT + ti];
            return ti + NT * (R + kk) < nv ? v : neg_inf16(sizeof(LT));
        };
        float m;
        if constexpr (IMAX) {                                  // (see k_q1_stats)
            s16x2 pm = {(short)-32768, (short)-32768};
#pragma unroll
            for (int j = 0; j < R; j++) {
                pm = __builtin_elementwise_max(pm, as_s16x2(x[j].x));
                pm = __builtin_elementwise_max(pm, as_s16x2(x[j].y));
                pm = __builtin_elementwise_max(pm, as_s16x2(x[j].z));
                pm = __builtin_elementwise_max(pm, as_s16x2(x[j].w));
            }
#pragma unroll
            for (int kk = 0; kk < L; kk++) {
                const u32x4 v = slot(kk);
                pm = __builtin_elementwise_max(pm, as_s16x2(v.x));
                pm = __builtin_elementwise_max(pm, as_s16x2(v.y));
                pm = __builtin_elementwise_max(pm, as_s16x2(v.z));
                pm = __builtin_elementwise_max(pm, as_s16x2(v.w));
            }
            const int li = pm.x > pm.y ? (int)pm.x : (int)pm.y;
            const int wi = (int)wave_reduce((uint32_t)li, [](uint32_t a, uint32_t b) {
                return (uint32_t)((int)a > (int)b ? (int)a : (int)b);
            });
            if (lane == 0) smaxi[w] = wi;
            if (!DEC && tid == 0) sps = 0;
            __syncthreads();
            int bi = smaxi[0];
#pragma unroll
            for (int i = 1; i < NW; i++) bi = smaxi[i] > bi ? smaxi[i] : bi;
            if constexpr (GROUP)                               // the int max of all segments
                bi = (int)group_combine((uint32_t)bi, [](uint32_t a, uint32_t b) { return (int)a > (int)b ? a : b; });
            if (bi >= 0 && bi <= 0x7F80) {                    // block-uniform (GROUP: the same in every segment)
                m = __uint_as_float((uint32_t)bi << 16);
            } else {
                float mx = -INFINITY;
#pragma unroll
                for (int j = 0; j < R; j++)
#pragma unroll
                    for (int e = 0; e < N; e++) mx = fmaxf(mx, logit_at<LT>(x[j], e));
#pragma unroll
                for (int kk = 0; kk < L; kk++) {
                    const u32x4 v = slot(kk);
#pragma unroll
                    for (int e = 0; e < N; e++) mx = fmaxf(mx, logit_at<LT>(v, e));
                }
                mx = wave_max_f32(mx);
                if (lane == 0) smax[w] = mx;
                __syncthreads();
                m = smax[0];
#pragma unroll
                for (int i = 1; i < NW; i++) m = fmaxf(m, smax[i]);
                if constexpr (GROUP)
                    m = __uint_as_float(group_combine(__float_as_uint(m), [](uint32_t a, uint32_t b) { return f32_max_bits(a, b); }));
            }
        } else {
            float mx = -INFINITY;
#pragma unroll
            for (int j = 0; j < R; j++)
#pragma unroll
                for (int e = 0; e < N; e++) mx = fmaxf(mx, logit_at<LT>(x[j], e));
#pragma unroll
            for (int kk = 0; kk < L; kk++) {
                const u32x4 v = slot(kk);
#pragma unroll
                for (int e = 0; e < N; e++) mx = fmaxf(mx, logit_at<LT>(v, e));
            }
            mx = wave_max_f32(mx);
            if (lane == 0) smax[w] = mx;
            if (!DEC && tid == 0) sps = 0;
            __syncthreads();
            m = smax[0];
#pragma unroll
            for (int i = 1; i < NW; i++) m = fmaxf(m, smax[i]);
            if constexpr (GROUP)
                m = __uint_as_float(group_combine(__float_as_uint(m), [](uint32_t a, uint32_t b) { return f32_max_bits(a, b); }));
        }
        const bool fast = q1_fast_row(m);
        const float c = q1_c(m);
        uint64_t tot = 0, lo = 0;
        int jl = 0;
        if (!DEC) {
            const int64_t s = sym[(t0 + r / B) * B + r % B];
            const int sc = (int)(s < 0 ? 0 : (s > V ? V : s));
            int sfull = sc / N;
            const int sr = sc - sfull * N;
            sfull -= vofs;                                     // GROUP: < 0 / >= nv: another segment's
            const int sfc = sfull < 0 ? 0 : (sfull > nv ? nv : sfull);
            const int js = sfull / NT, so = sfull - js * NT;  // vector js of thread so holds s
            jl = sfc > ti ? (sfc - ti + NT - 1) / NT : 0;      // this thread's vectors below it: j < jl
            if (sfull >= 0 && sfull < nv && w == so / 64 && js < R + L) {   // that thread's wave (uniform): split the
                u32x4 v = x[0];                                // vector once, before pass 2
#pragma unroll
                for (int j = 1; j < R; j++)
                    if (j == js) v = x[j];                     // (js uniform: scalar branches)
                if (L > 0 && js >= R) v = slot(js - R);
                uint32_t pl = 0, ps = 0;
#pragma unroll
                for (int e = 0; e < N; e++) {
                    const uint32_t q = q1_rep_at(tabr, q1_j(logit_at<LT>(v, e), c), loff);
                    pl += e < sr ? q : 0;
                    ps += e == sr ? q : 0;
                }
                const bool own = ti == so;
                lo = own ? pl : 0;
                if (own) sps = ps;
            }
        }
        if (sizeof(LT) == 2) {                                 // re-unpack in pass 2 (see k_q1_stats)
#pragma unroll
            for (int j = 0; j < R; j++) asm volatile("" : "+v"(x[j]));
        }
        // pass 2: lane sums of 8 vectors at a time in 32 bits (entries <= 2^24, at most 64
        // of them), folded into 64 bits per batch; DEC: the batch's 8 group totals.
        // Vectors past the row are summed too (tab0 each logit) and taken off after.
        // rolling prefetch: once vector j is summed its registers load vector j of the
        // block's next row, so that row streams in while this one is quantised (without
        // it a CU alternated a load phase and a compute phase: 61 vs 71 % of peak at bf16
        // Qwen2, profiles/r03/wide1/)
        const __amdgpu_buffer_rsrc_t rsn = rsrc(r + stride);
        // The fast / capped choice is a branch per batch around the sums only, with the
        // loads after it: with the whole pass 2 duplicated per branch, the next row's
        // registers met from two paths and the allocator spilled them (134-208 VGPRs).
        // Batches wholly past the row (NT j0 >= nv, uniform) skip their sums; their loads
        // are still issued (past the row they touch no memory) so that the registers
        // never meet from two paths.
        auto batch = [&](int j0) {
            uint32_t sv[8];
            const bool live = NT * j0 < nv;
            if (live && fast) {
#pragma unroll
                for (int u = 0; u < 8; u++) sv[u] = q1_vec_sum<LT>(x[j0 + u], c, true, tabr, loff);
            } else if (live) {
#pragma unroll
                for (int u = 0; u < 8; u++) sv[u] = q1_vec_sum<LT>(x[j0 + u], c, false, tabr, loff);
            } else {
#pragma unroll
                for (int u = 0; u < 8; u++) sv[u] = 0;
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 8; u++) x[j0 + u] = load_vec(rsn, j0 + u);
            if (!live) return;
            if constexpr (DEC) {
                // group (w + 8 j) = vectors [64 (w + 8 j), +64): wave w's vector j
                uint64_t gsum = wave_multi_sum32<8>(sv);        // lane l < 8: vector j0 + q_index<8>(l)
                if (lane < 8) {
                    // (the lane index fresh here: hoisted, the 7 batches' bin addresses spilled and
                    //  their reloads' vmcnt(0) drained the rolling prefetch)
                    const int grp = w + NW * (j0 + q_index<8>(lane_fresh())), past = (grp + 1) * 64 - nv;
                    if (past > 0 && past < 64) gsum -= (uint64_t)past * N * tab0;   // the row's last group
                    // (GROUP: segment group grp is the row's group vofs / 64 + grp; split is a multiple of 64)
                    if (grp * 64 < nv) atomicAdd(&bins[chunk_of(vofs / 64 + grp)], (unsigned long long)gsum);
                }
            } else {
                uint32_t bt = 0, bl = 0;
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    bt += sv[u];
                    bl += j0 + u < jl ? sv[u] : 0;
                }
                asm volatile("" : "+v"(bt), "+v"(bl));          // folded here, not sunk to the row's end
                tot += bt;
                lo += bl;
            }
        };
#pragma unroll
        for (int j0 = 0; j0 < R; j0 += 8) { batch(j0); __builtin_amdgcn_sched_barrier(0); }
        // the slot vectors, 8 at a time; each slot refilled with the next row's vector once
        // this wave's reads of it are done
        if constexpr (L > 0) {
            const bool nxt = r + stride < rows;                // uniform
            const LT *nrw = nxt ? row_of(r + stride) : lg;
#pragma unroll
            for (int k0 = 0; k0 < L; k0 += 8) {
                uint32_t sv[8];
                if (fast) {
#pragma unroll
                    for (int u = 0; u < 8; u++) sv[u] = k0 + u < L ? q1_vec_sum<LT>(slot(k0 + u), c, true, tabr, loff) : 0;
                } else {
#pragma unroll
                    for (int u = 0; u < 8; u++) sv[u] = k0 + u < L ? q1_vec_sum<LT>(slot(k0 + u), c, false, tabr, loff) : 0;
                }
                __builtin_amdgcn_s_waitcnt(0xc07f);            // lgkmcnt(0): the slot reads are done
                if (nxt) {
#pragma unroll
                    for (int u = 0; u < 8; u++)
                        if (k0 + u < L) ld_slot(nrw, k0 + u, ti, nv);
                }
                __builtin_amdgcn_sched_barrier(0);
                const int j0 = R + k0;
                if constexpr (DEC) {
                    uint64_t gsum = wave_multi_sum32<8>(sv);
                    if (lane < 8) {
                        const int grp = w + NW * (j0 + q_index<8>(lane_fresh())), past = (grp + 1) * 64 - nv;
                        if (past > 0 && past < 64) gsum -= (uint64_t)past * N * tab0;
                        if (grp * 64 < nv) atomicAdd(&bins[chunk_of(vofs / 64 + grp)], (unsigned long long)gsum);
                    }
                } else {
                    uint32_t bt = 0, bl = 0;
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        bt += sv[u];
                        bl += j0 + u < jl ? sv[u] : 0;
                    }
                    asm volatile("" : "+v"(bt), "+v"(bl));
                    tot += bt;
                    lo += bl;
                }
            }
        }
        if (!DEC) {
            const uint64_t t64 = wave_sum_u64(tot), l64 = wave_sum_u64(lo);
            if (lane == 0) { ssum[w][0] = t64; ssum[w][1] = l64; }
        }
        __syncthreads();
        if (DEC) {
            if (w == 0) {
                if constexpr (GROUP) {                         // into the zeroed chunk totals
                    const uint64_t v = bins[lane] + (pok ? 0 : kGroupPoison);
                    if (v) group_add(&chunks[r * 64 + lane], v);
                    if (lane == 0 && hh == 0) mrow[r] = m;
                } else {
                    chunks[r * 64 + lane] = bins[lane];
                    if (lane == 0) mrow[r] = m;
                }
                bins[lane] = 0;
            }
        } else if (tid == 0) {
            uint64_t T = 0, Ls = 0;
#pragma unroll
            for (int i = 0; i < NW; i++) { T += ssum[i][0]; Ls += ssum[i][1]; }
            // vectors of the live batches (L > 0: rows past the registers, every batch live)
            const int nsum = L > 0 ? NT * (R + L) : 8 * NT * ((nv + 8 * NT - 1) / (8 * NT));
            T -= (uint64_t)(nsum - nv) * N * tab0;             // those past the row
            if constexpr (GROUP) {                              // the segments' partials add up
                RowStats *o = out + r;                         // (zeroed; inv_tot 0: the coder divides)
                group_add(&o->tot, T + (pok ? 0 : kGroupPoison));
                group_add(&o->lo, Ls);
                group_add(&o->hi, Ls + sps);
                if (hh == 0) __hip_atomic_store(&o->minp, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                RowStats st;
                st.lo = Ls;
                st.hi = Ls + sps;
                st.tot = T;
                st.minp = 1;
                st.inv_tot = 1.0 / (double)T;
                st.pad = 0;
                out[r] = st;
            }
        }
    }
    if constexpr (L > 0) {
        __builtin_amdgcn_s_waitcnt(0);                         // no LDS-DMA outlives the block
        asm volatile("" ::: "memory");
    }
}
constexpr int kQ1WideR = 40;
constexpr int kQ1WideMaxVec = 512 * kQ1WideR;                  // registers only
constexpr int kQ1WideL = 11;                                   // + LDS slots (the 32-copy table beside them)
constexpr int kQ1WideSlotMaxVec = 512 * (kQ1WideR + kQ1WideL);

// k_q1_decode: one wave per stream, sequential over a chunk of steps, from the
// chunk totals of k_q1_stats: per step it finds the chunk holding
// floor((x-l)*T/w), re-quantises only that chunk's logits and scans them to the
// symbol, then renormalises as A_from_bin does (decode_advance).  A chunk's groups
// are loaded up to 4 at once and re-quantised one by one until the crossing (round 4:
// c4 7.23 -> 6.89, Qwen2 7.28 -> 6.79 us/step, profiles/r04/q1dec/; round 2 had
// re-quantised every loaded group, which measured no faster: with 16 stream-waves per
// CU the step is bound by their issue).
// GC: the groups per chunk when known at compile time (1..8; 0 = G at run time): one
// group (rows of <= 4096 vectors, the c3 shape) compiles to one straight-line pass
// instead of four unrolled copies inside a loop.
template <typename LT, int GC = 0, bool SMALL = true>
__global__ LAC_DEC_BOUNDS void k_q1_decode(const LT *__restrict__ lg, int64_t step_stride, int64_t stream_stride,
                                           int64_t t0, int64_t nsteps, int64_t V, int prec, uint32_t xsh,
                                           int64_t Garg, const uint64_t *__restrict__ chunks,
                                           const float *__restrict__ mrow, DecState *states, const uint8_t *bits,
                                           uint64_t stride, const uint64_t *nbits, int32_t *sym_out, int64_t B) {
    // (one shared table copy: 8 or 16 lane-interleaved copies against the gathers' bank
    // conflicts measured no faster, profiles/r04/q1dec/)
    const int64_t G = GC ? GC : Garg;
    constexpr int GPF = GC ? GC : 4;                            // group loads in flight
    __shared__ uint32_t tab[LAC_Q1_TAB_SIZE];
    q1_load_tab(tab, xsh);
    constexpr int N = LogitN<LT>::N;
    const int lane = (int)lane_id();
    // (round 4) the stream and its decoder state wave-uniform (SGPRs): the serial chain
    // -- targets, ranges, renormalisation, the determined test -- runs on the scalar
    // unit with uniform branches, its quotients by div_small (q1 totals are <= 2^(prec-1),
    // so at prec <= 50 every quotient is below 2^50); the vector unit keeps the chunk
    // scan and the re-quantisation of one 64-vector group per search round
    const int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + wave_in_block();
    if (b >= B) return;
    DecState st = states[b];
    dec_state_uniform(st);
    const uint8_t *mybits = bits + b * stride;
    const uint64_t mynbits = rfl_u64(nbits[b]);
    const int64_t nvec = V / N;
    const bool small = SMALL;                                   // (the host passes prec <= 50)
    uint64_t next = nsteps > 0 ? chunks[b * 64 + lane] : 0;
    float mnext = nsteps > 0 ? mrow[b] : 0.f;
    // (as k_decode_lean) a 32-bit step counter, running row pointers, and the symbols
    // collected one per lane and stored once per 64 steps
    const int32_t n32 = (int32_t)nsteps;                        // (<= chunk_steps)
    const LT *rowp = lg + t0 * step_stride + b * stream_stride;
    int32_t *outv = sym_out + (t0 + lane) * B + b;              // lane j: step 64k + j
    int32_t sbuf = -1;
    int32_t i = 0;
    for (; i < n32; i++) {
        dec_state_uniform(st);                                 // (the loop's phis are not seen as uniform)
        const int64_t r = (int64_t)i * B + b;
        const uint64_t mine = next;
        const float mcur = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, mnext)));
        if (i + 1 < n32) {                                     // prefetch: independent of the state
            next = chunks[(r + B) * 64 + lane];
            mnext = mrow[r + B];
        }
        const LT *row = rowp;
        rowp += step_stride;
        if (st.err) {
            if (lane == (i & 63)) sbuf = -1;
            if ((i & 63) == 63) {
                *outv = sbuf;
                outv += B * 64;
            }
            continue;
        }
        const BitWin win = bit_window(mybits, mynbits, st.pos);    // in flight during the search
        const float c = q1_c(mcur);
        const uint64_t incl = wave_incl_scan_u64(mine);
        const uint64_t T = readlane_u64(incl, 63);
        int err = 0;
        int64_t s = -1;
        const int64_t l = st.l, h = st.h, x = st.x;
        if (x < l || x > h) err = LAC_E_DECODE_RANGE;
        const uint64_t w = (uint64_t)(h - l + 1), v = (uint64_t)(x - l);
        if (!err && T > w) err = LAC_E_TABLE;                  // fudged (minp 1): impossible by the choice of k
        if (!err) {
            const uint64_t past = st.pos > mynbits ? st.pos - mynbits : 0;
            const int u = past < (uint64_t)prec ? (int)past : prec;
            const uint64_t vh = v + ((1ull << u) - 1);
            uint64_t tgt, thi;
            if (small) {
                const double iw = recip(w);
                tgt = div_small_u(v, T, 0, w, iw);
                thi = vh == v ? tgt : (vh < w ? div_small_u(vh, T, 0, w, iw) : 0);
            } else {
                div_pair(v, vh < w ? vh : 0, T, 0, w, recip(w), &tgt, &thi);
            }
            const uint64_t ex = incl - mine;
            const uint64_t mask = __ballot(ex <= tgt && tgt < incl);
            if (!mask) err = LAC_E_DECODE_RANGE;
            if (!err) {
                const int src = __ffsll((unsigned long long)mask) - 1;
                uint64_t cb = readlane_u64(ex, src);
                const int64_t cv0 = (int64_t)src * G * 64;
                // a chunk whose total is below 2^32 (nearly all) scans its groups in 32 bits
                const bool narrow = readlane_u64(mine, src) < (1ull << 32);
                // the crossing lane by ballot, as scan_chunk (entries <= tgt are a prefix);
                // a lane's 8 (bf16) / 4 (f32) entries are <= 2^24 each, so its own prefix
                // runs in 32 bits and only the wave scan needs 64
                uint64_t lo_c = cb, hi_c = ~0ull, cnt = 0;
                bool found = false;
                // the chunk's groups, up to 4 loads in flight (clamped in-row indices), then
                // re-quantised and scanned one by one until the crossing
                for (int64_t g0 = 0; g0 < G && !found; g0 += GPF) {
                u32x4 xq[GPF];
#pragma unroll
                for (int u = 0; u < GPF; u++) {
                    const int64_t vi = cv0 + (g0 + u) * 64 + lane;
                    xq[u] = ld16(row, (g0 + u < G && vi < nvec) ? vi : nvec - 1, false);
                }
#pragma unroll
                for (int u = 0; u < GPF; u++) {
                    const int64_t g = g0 + u;
                    if (found || g >= G) break;
                    const int64_t vi = cv0 + g * 64 + lane;
                    const bool valid = vi < nvec;
                    const u32x4 xv = xq[u];
                    uint32_t loc[N], ls = 0;
#pragma unroll
                    for (int j = 0; j < N; j++) {
                        // looked up unconditionally (xv is a clamped in-row vector), masked
                        // after: a conditional lookup compiled to one exec-masked branch
                        // with its own LDS wait per entry
                        const uint32_t q = q1_val(logit_at<LT>(xv, j), c, tab);
                        ls += valid ? q : 0u;
                        loc[j] = ls;
                    }
                    const uint64_t in = narrow ? (uint64_t)wave_incl_scan_u32(ls) : wave_incl_scan_u64((uint64_t)ls);
                    const uint64_t exb = cb + in - ls;
                    const uint64_t m = __ballot(exb + ls > tgt);
                    if (m) {
                        const int L = __ffsll((unsigned long long)m) - 1;
                        // lane L: exb <= tgt < exb + ls, so tgt - exb fits 32 bits there
                        const uint32_t rel = (uint32_t)(tgt - exb);
                        uint32_t k = 0, lo = 0, hi = ~0u;
#pragma unroll
                        for (int j = 0; j < N; j++) {
                            const bool le = loc[j] <= rel;
                            k += le ? 1u : 0u;
                            lo = le ? loc[j] : lo;
                            hi = (!le && loc[j] < hi) ? loc[j] : hi;
                        }
                        const uint64_t eb = readlane_u64(exb, L);
                        cnt = (uint64_t)(g * 64 + L) * N + (uint64_t)__builtin_amdgcn_readlane((int)k, L);
                        lo_c = eb + (uint32_t)__builtin_amdgcn_readlane((int)lo, L);
                        hi_c = eb + (uint32_t)__builtin_amdgcn_readlane((int)hi, L);
                        found = true;
                    }
                    cb += readlane_u64(in, 63);
                }
                }
                if (!found) {
                    err = LAC_E_DECODE_RANGE;                  // corrupt state: tgt outside the chunk
                } else {
                    s = cv0 * N + (int64_t)cnt;
                    uint64_t a, bb;
                    if (small) {
                        div_small_u2(lo_c, hi_c, w, T - 1, T, recip(T), &a, &bb);
                    } else {
                        div_pair(lo_c, hi_c, w, T - 1, T, recip(T), &a, &bb);
                    }
                    const bool det = vh < w && thi < hi_c;
                    if (st.det && det) st.ndet++;
                    else st.det = 0;
                    err = decode_advance<true>(st, a, bb, win, mynbits, prec);
                }
            }
        }
        if (err) {
            st.err = err;
            st.err_step = st.nsym;
        }
        if (lane == (i & 63)) sbuf = err ? -1 : (int32_t)s;
        if ((i & 63) == 63) {
            *outv = sbuf;
            outv += B * 64;
        }
    }
    if (lane < (i & 63)) *outv = sbuf;
    if (lane == 0) states[b] = st;
}

// Materialise q1 tables (for parity checks and for callers that want them).
template <typename LT>
__global__ __launch_bounds__(256) void k_quantize_logits(const LT *__restrict__ lg, int64_t step_stride,
                                                         int64_t stream_stride, int64_t B, int64_t rows, int64_t V,
                                                         uint32_t xsh, uint32_t *__restrict__ out) {
    __shared__ uint32_t tab[LAC_Q1_TAB_SIZE];
    q1_load_tab(tab, xsh);
    constexpr int N = LogitN<LT>::N;
    const int lane = (int)lane_id();
    const int64_t r = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (r >= rows) return;
    const LT *row = lg + (r / B) * step_stride + (r % B) * stream_stride;
    const int64_t nvec = V / N;
    float mx = -INFINITY;
    for (int64_t vi = lane; vi < nvec; vi += 64) {
        const u32x4 x = ld16(row, vi, false);
#pragma unroll
        for (int j = 0; j < N; j++) mx = fmaxf(mx, logit_at<LT>(x, j));
    }
    const float c = q1_c(wave_max_f32(mx));
    uint32_t *o = out + r * V;
    for (int64_t vi = lane; vi < nvec; vi += 64) {
        const u32x4 x = ld16(row, vi, true);
#pragma unroll
        for (int j = 0; j < N; j++) o[vi * N + j] = q1_val(logit_at<LT>(x, j), c, tab);
    }
}

#include "lac_tail.h"

}  // namespace

// ====================================================================== C-ABI
struct lac_ctx {
    int device = 0, prec = 0, pmf_bits = 32;
    int64_t V = 0, B = 0;
    uint64_t cap_bits = 0, cap_words = 0;
    RowStats *stats = nullptr;
    EncState *enc = nullptr;
    DecState *dec = nullptr;
    TailState *tail = nullptr;          // decoder tail in the reference frame (lac_decode_tail_*)
    uint64_t *planeA = nullptr, *planeC = nullptr, *nbits = nullptr;
    uint64_t *own_planeA = nullptr, *own_nbits = nullptr;   // planeA / nbits unless lac_set_output redirects them
    const uint8_t *dbits = nullptr;
    uint64_t dstride = 0;
    const uint64_t *dnbits = nullptr;
    int mode = 0;                       // 0 encode, 1 decode
    int finished = 0;                   // nbits / planeA hold finished streams (a job, lac_encode_finish)
    int path = LAC_PATH_AUTO;           // encode kernel path (lac_set_option)
    int64_t fused_min_streams = 2048;   // AUTO: fused kernel from this many streams
    int64_t chunk_steps = 64;           // split path: steps per row-stats launch
    int dpath = LAC_PATH_AUTO;          // decode kernel path
    int64_t wave_decode_min_streams = 2048;   // measured: the stats path wins at 1024 streams
    int fine_decode = 1;                // one-wave decode: per-iteration totals (k_decode_wave_fine)
    int64_t block_decode_min_streams = 1536;  // AUTO below wave_decode_min_streams: block path from here
                                              // (measured after the serial-step rework: the stats path wins
                                              // at 4-128 and 288-1024 streams, block at 160-256 -- its
                                              // 16-wave groups fill the chip in one round up to 256
                                              // streams -- and at 1536; profiles/r01/decode_paths_v2/)
    int64_t block_window_lo = 160, block_window_hi = 256;   // AUTO: block path inside this window too --
                                              // one 16-wave group per stream fills the chip in one round
                                              // while streams <= CUs; set from the CU count at open
    int block_waves = 0;                // block path waves per stream (0 = by stream count)
    int mapping = LAC_MAP_CEIL;         // symbol_to_range flavour (lac_set_option)
    int term = LAC_TERM_FLUSH;          // stream termination flavour
    int cus = 256;                      // compute units (persistent grids)
    int q1_shape = 0;                   // logits stats block shape (0 auto; lac_set_option tuning)
    uint64_t *q1chunks = nullptr;       // logits / stats-path decode: [chunk_steps * B][64] chunk totals
    void *dmeta = nullptr;              // stats-path decode: [chunk_steps * B] DecRowMeta
    int64_t *dresume = nullptr;         //                    [B] first step k_decode_lean left
    void *lvpre = nullptr;              // lean decode: [lean_steps * B][V / VEC] uint32 vector CDF
    uint64_t *lchunk = nullptr;         //              [lean_steps * B][64] chunk bounds
    void *lmeta = nullptr;              //              [lean_steps * B] LeanMeta
    int64_t lean_steps = 0;             //              steps per launch the buffers hold
    int32_t *dprogress = nullptr;       //              [B] decoder progress for the prefetch helpers
    float *q1m = nullptr;               //                [chunk_steps * B] row maxima
    uint64_t *pxch = nullptr;           // paired row stats (shape 19): [2 * cus] maximum words
    int64_t xch_abort = -1;             // word of pxch holding the last row-group launch's abort flag
    // live kernel timing (lac_profile_enable): hipEvent pairs around launches
    bool prof = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> ev_used;   // kernel id, (start, stop)
    size_t ev_next = 0;
};

enum { KID_ROW_STATS = 0, KID_ENCODE = 1, KID_FINISH = 2, KID_DECODE = 3, KID_FUSED = 4, KID_DECODE_WAVE = 5,
       KID_Q1_STATS = 6, KID_Q1_DECODE = 7, KID_COUNT = 8 };
// the stats-path decode (k_dec_stats + k_decode_seq) reports under KID_DECODE

static hipEvent_t ev_get(lac_ctx *c) {
    if (c->ev_next == c->ev_pool.size()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        c->ev_pool.push_back(e);
    }
    return c->ev_pool[c->ev_next++];
}

// Brackets one launch with events on its stream when profiling is on.
struct ProfScope {
    lac_ctx *c;
    int kid;
    hipStream_t st;
    hipEvent_t a = nullptr, b = nullptr;
    ProfScope(lac_ctx *c_, int kid_, hipStream_t st_) : c(c_), kid(kid_), st(st_) {
        if (c->prof && kid >= 0) {
            a = ev_get(c);
            b = ev_get(c);
            if (a && b) (void)hipEventRecord(a, st);
        }
    }
    ~ProfScope() {
        if (c->prof && a && b) {
            (void)hipEventRecord(b, st);
            c->ev_used.push_back({kid, {a, b}});
        }
    }
};

static thread_local std::string g_err;

static int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
static int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIPCHK(x)                                                                          \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) return fail(LAC_E_HIP, "%s: %s", #x, hipGetErrorString(e_)); \
    } while (0)

#define CHECK_LAUNCH() HIPCHK(hipGetLastError())

static inline hipStream_t S(void *s) { return reinterpret_cast<hipStream_t>(s); }

template <typename E, int VEC>
static int encode_impl(lac_ctx *c, const E *pmf, int64_t step_stride, int64_t stream_stride, const int32_t *sym,
                       int64_t steps, uint64_t *trace, hipStream_t st, int flags) {
    const unsigned blocks = (unsigned)((c->B + kWavesPerBlock - 1) / kWavesPerBlock);
    const bool fused = c->path == LAC_PATH_FUSED || (c->path == LAC_PATH_AUTO && c->B >= c->fused_min_streams);
    if (fused) {
        ProfScope ps(c, KID_FUSED, st);
        k_encode_fused<E, VEC><<<(unsigned)((c->B + kStreamWaves - 1) / kStreamWaves), 64 * kStreamWaves, 0, st>>>(
            pmf, step_stride, stream_stride, sym, c->B, 0, steps, c->V, c->prec, c->enc, c->planeA, c->planeC,
            c->cap_words, trace, c->nbits, flags, c->mapping, c->term);
        CHECK_LAUNCH();
        return LAC_OK;
    }
    if (flags & kReset) {
        k_enc_reset<<<(unsigned)((c->B + 255) / 256), 256, 0, st>>>(c->enc, c->B, c->prec);
        CHECK_LAUNCH();
    }
    for (int64_t t0 = 0; t0 < steps; t0 += c->chunk_steps) {
        const int64_t n = (steps - t0) < c->chunk_steps ? (steps - t0) : c->chunk_steps;
        const int64_t rows = n * c->B;
        {
            ProfScope ps(c, KID_ROW_STATS, st);
            k_row_stats<E, VEC><<<(unsigned)((rows + kWavesPerBlock - 1) / kWavesPerBlock), 64 * kWavesPerBlock, 0,
                                  st>>>(pmf, step_stride, stream_stride, sym, c->B, rows, c->V, t0, c->stats);
        }
        CHECK_LAUNCH();
        {
            ProfScope ps(c, KID_ENCODE, st);
            k_encode<E><<<blocks, 64 * kWavesPerBlock, 0, st>>>(c->stats, sym, c->B, t0, n, pmf, step_stride,
                                                                stream_stride, c->V, c->prec, c->enc, c->planeA,
                                                                c->planeC, c->cap_words, trace, c->mapping, true);
        }
        CHECK_LAUNCH();
    }
    if (flags & kFinish) {
        ProfScope ps(c, KID_FINISH, st);
        k_finish<<<(unsigned)((c->B + 255) / 256), 256, 0, st>>>(c->enc, c->planeA, c->planeC, c->cap_words, c->B,
                                                                 c->prec, c->nbits, c->term);
        CHECK_LAUNCH();
    }
    return LAC_OK;
}

static int encode_dispatch(lac_ctx *c, const void *pmf_dev, int64_t step_stride, int64_t stream_stride,
                           const int32_t *sym_dev, int64_t steps, uint64_t *trace_dev, void *stream, int flags) {
    if (!c || (steps > 0 && (!pmf_dev || !sym_dev))) return fail(LAC_E_ARG, "NULL argument");
    if (steps < 0 || step_stride < 0 || stream_stride < 0) return fail(LAC_E_ARG, "negative size/stride");
    if (steps == 0 && !flags) return LAC_OK;
    HIPCHK(hipSetDevice(c->device));
    c->mode = 0;
    hipStream_t st = S(stream);
    const uintptr_t p = (uintptr_t)pmf_dev;
    if (c->pmf_bits == 32) {
        const bool vec = (p % 16 == 0) && c->V % 4 == 0 && step_stride % 4 == 0 && stream_stride % 4 == 0;
        return vec ? encode_impl<uint32_t, 4>(c, (const uint32_t *)pmf_dev, step_stride, stream_stride, sym_dev, steps,
                                              trace_dev, st, flags)
                   : encode_impl<uint32_t, 1>(c, (const uint32_t *)pmf_dev, step_stride, stream_stride, sym_dev, steps,
                                              trace_dev, st, flags);
    }
    const bool vec = (p % 16 == 0) && c->V % 2 == 0 && step_stride % 2 == 0 && stream_stride % 2 == 0;
    return vec ? encode_impl<uint64_t, 2>(c, (const uint64_t *)pmf_dev, step_stride, stream_stride, sym_dev, steps,
                                          trace_dev, st, flags)
               : encode_impl<uint64_t, 1>(c, (const uint64_t *)pmf_dev, step_stride, stream_stride, sym_dev, steps,
                                          trace_dev, st, flags);
}

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

static int ensure_chunk_buffers(lac_ctx *c) {
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
    // k_decode_lean: u32 tables, prec <= 50, chunks of at most 4 iterations (V <= 65536); its
    // buffers hold up to 64 MB of vector CDFs, so its launches take at most that many steps
    const int64_t nvec = c->V / VEC, nit = (nvec + 63) / 64;
    const int64_t CI = nit ? (nit + 63) / 64 : 1;
    // (u64 tables: totals >= 2^32.)  Only for the fewest streams: the stats pass writes a
    // quarter of the rows' bytes more (the vector CDF), which costs more than the shorter
    // chain saves once enough streams run side by side (same box, V=32000: B=4 1.36 vs
    // 2.66 us/step, 64 3.41 vs 3.96, 128 5.39 vs 5.26, 512 18.0 vs 13.3, 1024 34.1 vs 22.8;
    // profiles/r04/lean/fewstreams/)
    const bool lean = LAC_LEAN && sizeof(E) == 4 && c->prec <= 50 && CI <= 4 && nvec > 0 && c->B <= kLeanMaxStreams;
    int64_t cs = c->chunk_steps;
    if (lean) {
        const int64_t per = c->B * nvec * (int64_t)sizeof(uint32_t);
        const int64_t fit = ((int64_t)64 << 20) / per;
        const int64_t ls = fit < 64 ? 64 : fit / 64 * 64;
        cs = ls < cs ? ls : cs;
        if (c->lean_steps < cs) {
            (void)hipFree(c->lvpre);
            (void)hipFree(c->lchunk);
            (void)hipFree(c->lmeta);
            c->lvpre = nullptr;
            c->lchunk = nullptr;
            c->lmeta = nullptr;
            c->lean_steps = 0;
            HIPCHK(hipMalloc(&c->lvpre, sizeof(uint32_t) * cs * c->B * nvec));
            HIPCHK(hipMalloc(&c->lchunk, sizeof(uint64_t) * 64 * cs * c->B));
            HIPCHK(hipMalloc(&c->lmeta, sizeof(LeanMeta) * cs * c->B));
            c->lean_steps = cs;
        }
        if (!c->dresume) HIPCHK(hipMalloc(&c->dresume, sizeof(int64_t) * c->B));
    }
    // prefetching helper workgroups for the fewest streams (kLeanHelpers per stream, dealt
    // to the stream's XCD)
    const bool help = lean && LAC_LEAN_HELP && c->B <= kLeanHelpMaxStreams;
    const int64_t B8 = (c->B + 7) & ~(int64_t)7;
    const unsigned lean_blocks = (unsigned)(help ? B8 * (1 + kLeanHelpers) : c->B);
    if (help && !c->dprogress) HIPCHK(hipMalloc(&c->dprogress, sizeof(int32_t) * c->B));
    for (int64_t t0 = 0; t0 < steps; t0 += cs) {
        const int64_t n = (steps - t0) < cs ? (steps - t0) : cs;
        const int64_t rows = n * c->B;
        ProfScope ps(c, KID_DECODE, st);
        const unsigned sblocks = (unsigned)((rows + kWavesPerBlock - 1) / kWavesPerBlock);
        if (lean) {
            k_dec_stats<E, VEC, true><<<sblocks, 64 * kWavesPerBlock, 0, st>>>(
                pmf, step_stride, stream_stride, c->B, rows, c->V, t0, c->q1chunks, (DecRowMeta *)c->dmeta,
                (uint32_t *)c->lvpre, c->lchunk, (LeanMeta *)c->lmeta);
            CHECK_LAUNCH();
            if (help) HIPCHK(hipMemsetAsync(c->dprogress, 0, sizeof(int32_t) * c->B, st));
#define LAC_LEAN_K(CIM)                                                                                          \
    k_decode_lean<E, VEC, CIM><<<lean_blocks, 64, 0, st>>>(                                                    \
        pmf, step_stride, stream_stride, t0, n, c->V, c->prec, (const uint32_t *)c->lvpre, c->lchunk,          \
        (const LeanMeta *)c->lmeta, c->dec, c->dbits, c->dstride, c->dnbits, out, c->B, c->mapping, c->dresume, \
        help ? c->dprogress : nullptr)
            switch (CI) {
            case 1: LAC_LEAN_K(1); break;
            case 2: LAC_LEAN_K(2); break;
            case 3: LAC_LEAN_K(3); break;
            default: LAC_LEAN_K(4); break;
            }
#undef LAC_LEAN_K
            CHECK_LAUNCH();
        } else {
            k_dec_stats<E, VEC><<<sblocks, 64 * kWavesPerBlock, 0, st>>>(
                pmf, step_stride, stream_stride, c->B, rows, c->V, t0, c->q1chunks, (DecRowMeta *)c->dmeta);
            CHECK_LAUNCH();
        }
        k_decode_seq<E, VEC><<<blocks, 64 * kWavesPerBlock, 0, st>>>(
            pmf, step_stride, stream_stride, t0, n, c->V, c->prec, c->q1chunks, (const DecRowMeta *)c->dmeta, c->dec,
            c->dbits, c->dstride, c->dnbits, out, c->B, c->mapping, lean ? c->dresume : nullptr);
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

// ---- logits path host side
static int q1_shift(lac_ctx *c, uint32_t *xsh) {
    int cl = 0;
    while (((int64_t)1 << cl) < c->V) cl++;                      // ceil(log2 V)
    int k = c->prec - 1 - cl;
    if (k > LAC_Q1_KMAX) k = LAC_Q1_KMAX;
    if (k < 1) return fail(LAC_E_PREC, "prec %d leaves no q1 precision for vocab %lld", c->prec, (long long)c->V);
    *xsh = (uint32_t)(LAC_Q1_KMAX - k);
    return LAC_OK;
}

static int logits_check(lac_ctx *c, const void *lg, int type, int64_t step_stride, int64_t stream_stride,
                        int64_t steps) {
    if (type != LAC_LOGITS_BF16 && type != LAC_LOGITS_F32) return fail(LAC_E_ARG, "logit type %d", type);
    if (steps < 0 || step_stride < 0 || stream_stride < 0) return fail(LAC_E_ARG, "negative size/stride");
    const int n = type == LAC_LOGITS_BF16 ? 8 : 4;
    if (steps > 0 && ((uintptr_t)lg % 16 || c->V % n || step_stride % n || stream_stride % n))
        return fail(LAC_E_ARG, "logits rows must be 16-byte aligned with vocab and strides multiples of %d", n);
    if (c->mapping != LAC_MAP_CEIL || c->term != LAC_TERM_FLUSH)
        return fail(LAC_E_STATE, "the logits path codes with the CDFPredictor mapping and flush termination");
    return LAC_OK;
}

static int64_t q1_groups_per_chunk(int64_t nvec) {                // 64-vector groups per decode chunk
    const int64_t groups = (nvec + 63) / 64;
    return groups <= 64 ? 1 : (groups + 63) / 64;
}

struct Q1Args {
    const void *lg;
    int64_t ss, bs;
    const int32_t *sym;
    int64_t rows, t0;
    uint32_t xsh;
};

template <typename LT, int RW, int R, bool DEC, bool MULTI, bool PF, int NWB = kQ1Waves>
static int q1_stats_launch(lac_ctx *c, const Q1Args &a, hipStream_t st, const uint64_t *gate = nullptr) {
    static int per_cu = 0;                                       // resident blocks per CU (occupancy API)
    if (!per_cu) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_q1_stats<LT, RW, R, DEC, MULTI, PF, NWB>, 64 * NWB,
                                                         0) != hipSuccess ||
            n < 1)
            n = 1;
        per_cu = n;
    }
    constexpr int NR = NWB / RW;
    const int64_t need = (a.rows + NR - 1) / NR, cap = (int64_t)c->cus * per_cu;
    const unsigned grid = (unsigned)(need < cap ? need : cap);
    const int64_t nvec = c->V / LogitN<LT>::N;
    ProfScope ps(c, gate ? -1 : KID_Q1_STATS, st);            // (a gated repair launch is not profiled)
    k_q1_stats<LT, RW, R, DEC, MULTI, PF, NWB><<<grid, 64 * NWB, 0, st>>>(
        (const LT *)a.lg, a.ss, a.bs, a.sym, c->B, a.rows, c->V, a.t0, a.xsh, q1_groups_per_chunk(nvec), c->stats,
        c->q1chunks, c->q1m, gate);
    CHECK_LAUNCH();
    return LAC_OK;
}

template <typename LT, bool DEC>
static int q1_wide_launch(lac_ctx *c, const Q1Args &a, hipStream_t st) {
    const int64_t cap = (int64_t)c->cus;                         // one 8-wave block per CU
    const unsigned grid = (unsigned)(a.rows < cap ? a.rows : cap);
    const int64_t nvec = c->V / LogitN<LT>::N;
    ProfScope ps(c, KID_Q1_STATS, st);
    if (nvec <= kQ1WideMaxVec)
        k_q1_stats_wide<LT, kQ1WideR, DEC><<<grid, 512, 0, st>>>(
            (const LT *)a.lg, a.ss, a.bs, a.sym, c->B, a.rows, c->V, a.t0, a.xsh, q1_groups_per_chunk(nvec), c->stats,
            c->q1chunks, c->q1m, nullptr, 0, 1, 0);
    else                                                         // rows past the registers: + LDS slots
        k_q1_stats_wide<LT, kQ1WideR, DEC, false, kQ1WideL><<<grid, 512, 0, st>>>(
            (const LT *)a.lg, a.ss, a.bs, a.sym, c->B, a.rows, c->V, a.t0, a.xsh, q1_groups_per_chunk(nvec), c->stats,
            c->q1chunks, c->q1m, nullptr, 0, 1, 0);
    CHECK_LAUNCH();
    return LAC_OK;
}

template <typename LT, bool DEC, int REP, int LASTN, int NT>
static int q1_rl_kernel(lac_ctx *c, const Q1Args &a, hipStream_t st) {
    constexpr int NRB = 1024 / NT;
    const int64_t need = (a.rows + NRB - 1) / NRB, cap = (int64_t)c->cus;   // one 16-wave block per CU
    const unsigned grid = (unsigned)(need < cap ? need : cap);
    const int64_t nvec = c->V / LogitN<LT>::N;
    ProfScope ps(c, KID_Q1_STATS, st);
    k_q1_stats_rl<LT, DEC, REP, LASTN, NT><<<grid, 1024, 0, st>>>(
        (const LT *)a.lg, a.ss, a.bs, a.sym, c->B, a.rows, c->V, a.t0, a.xsh, q1_groups_per_chunk(nvec), c->stats,
        c->q1chunks, c->q1m, nullptr, 0, 1, 0);
    CHECK_LAUNCH();
    return LAC_OK;
}

// Grouped row stats (shapes 19 / 20 / 21): a row in kg segments of `split` vectors
// (a multiple of 64; the last one the rest), one per row slot of the rl kernel
// with NRB = 1 / 2 / 4 rows per block; every segment must fit its slot -- the
// 16-copy form (16064 / 8000 / 4032 vectors) or the 8-copy form (16384 / 8192 /
// 4096).  Decode has no 16-copy form at NRB = 4 (LDS: its group totals).
constexpr int kQ1MaxSeg = 16;                    // segments per row (lanes polling partners)
struct Q1Group {
    int k = 0, split = 0, nrb = 1;
    bool rep16 = false;
    double score = 0;
};
static int64_t q1_slot_cap(int nrb, bool rep16) {
    if (nrb == 1) return rep16 ? kRLTrimMaxVec : 16384;
    if (nrb == 2) return rep16 ? 15 * 512 + 320 : 8192;
    return rep16 ? 15 * 256 + 192 : 4096;
}
// the fewest segments of this form; score = the row's share of its slots' capacity
// (the bytes a CU keeps in flight) x the share of the XCD's slots in use
static bool q1_group_form(lac_ctx *c, int64_t nvec, int nrb, bool rep16, Q1Group *g) {
    const int64_t ngrp = (nvec + 63) / 64, lim = q1_slot_cap(nrb, rep16), spx = (int64_t)(c->cus / 8) * nrb;
    for (int k = 2; k <= kQ1MaxSeg && k <= spx; k++) {
        const int64_t sp = 64 * ((ngrp + k - 1) / k), last = nvec - (k - 1) * sp;
        if (last > 0 && sp <= lim && last <= lim) {
            g->k = k;
            g->split = (int)sp;
            g->nrb = nrb;
            g->rep16 = rep16;
            g->score = (double)nvec / (k * (16384.0 / nrb)) * (double)((spx / k) * k) / (double)spx;
            return true;
        }
    }
    return false;
}
// nrb = 0: the best-scoring form (ties: the first, i.e. fewer rows per block and the
// 16-copy form); decode's 8-copy forms score 5 % lower (q1_rl_rep16: its lookups
// are the bound there; encode measured the same either way), and bf16 encode's
// 25 % lower: with the group logic they spill 29-32 VGPRs at the 128 cap (the
// 16-copy ones none), and the round-2 pair form at V = 262144 ran at 59 % of peak
// against 78 % for V = 256000's 16-copy halves
static bool q1_group(lac_ctx *c, int64_t nvec, bool dec, bool bf16, int nrb, Q1Group *best) {
    bool any = false;
    for (int n : {1, 2, 4}) {
        if (nrb && n != nrb) continue;
        for (int rep16 = 1; rep16 >= 0; rep16--) {
            if (dec && n == 4 && rep16) continue;
            Q1Group g;
            if (!q1_group_form(c, nvec, n, rep16 != 0, &g)) continue;
            if (!rep16) g.score *= dec ? 0.95 : bf16 ? 0.75 : 1.0;
            if (!any || g.score > best->score + 1e-9) *best = g;
            any = true;
        }
    }
    return any;
}

template <typename LT, bool DEC, int REP, int LASTN, int NT>
static int q1_group_kernel(lac_ctx *c, const Q1Args &a, hipStream_t st, const Q1Group &g) {
    constexpr int NRB = 1024 / NT;
    const int64_t nvec = c->V / LogitN<LT>::N;
    // (<= 4 rows per block) + the abort word
    if (!c->pxch) HIPCHK(hipMalloc(&c->pxch, sizeof(uint64_t) * (8 * (int64_t)c->cus + 1)));
    // rpx rows per XCD per round (all of the XCD's slots' worth, or all rows in one
    // round), on the fewest blocks that hold rpx * k slots; never more blocks than
    // CUs (one per CU: every partner resident at once)
    const int64_t spx = (int64_t)(c->cus / 8) * NRB, rcap = spx / g.k, rneed = (a.rows + 7) / 8;
    const int64_t rpx = rneed < rcap ? rneed : rcap;
    const unsigned grid = (unsigned)(8 * ((rpx * g.k + NRB - 1) / NRB));
    HIPCHK(hipMemsetAsync(c->pxch, 0, sizeof(uint64_t) * (2 * NRB * grid + 1), st));   // no stale sequence numbers,
                                                                                      // abort word clear
    // the segments add into zeroed outputs
    if (DEC) HIPCHK(hipMemsetAsync(c->q1chunks, 0, sizeof(uint64_t) * 64 * a.rows, st));
    else HIPCHK(hipMemsetAsync(c->stats, 0, sizeof(RowStats) * a.rows, st));
    {
        ProfScope ps(c, KID_Q1_STATS, st);
        k_q1_stats_rl<LT, DEC, REP, LASTN, NT, true><<<grid, 1024, 0, st>>>(
            (const LT *)a.lg, a.ss, a.bs, a.sym, c->B, a.rows, c->V, a.t0, a.xsh, q1_groups_per_chunk(nvec), c->stats,
            c->q1chunks, c->q1m, c->pxch, g.split, g.k, (int)rpx);
        CHECK_LAUNCH();
    }
    // repair: the tiled two-pass shape over the same rows, gated on the abort word
    // (its blocks exit at once when the groups completed: one small launch per job)
    const uint64_t *gate = c->pxch + 2 * NRB * grid;
    c->xch_abort = 2 * NRB * (int64_t)grid;
    if (DEC) return q1_stats_launch<LT, 16, 16, DEC, true, false, 16>(c, a, st, gate);            // shape 10
    if (sizeof(LT) == 4) return q1_stats_launch<LT, 16, 8, DEC, true, true, 16>(c, a, st, gate);  // shape 14
    return q1_stats_launch<LT, 8, 8, DEC, true, false>(c, a, st, gate);                            // shape 8
}

template <typename LT, bool DEC>
static int q1_stats_group_launch(lac_ctx *c, const Q1Args &a, hipStream_t st, const Q1Group &g) {
    if (g.nrb == 4) {
        if constexpr (!DEC)
            if (g.rep16) return q1_group_kernel<LT, DEC, 16, 192, 256>(c, a, st, g);
        return q1_group_kernel<LT, DEC, kRLRep, 256, 256>(c, a, st, g);
    }
    if (g.nrb == 2) {
        if (g.rep16) return q1_group_kernel<LT, DEC, 16, 320, 512>(c, a, st, g);
        return q1_group_kernel<LT, DEC, kRLRep, 512, 512>(c, a, st, g);
    }
    if (g.rep16) return q1_group_kernel<LT, DEC, 16, kRLLastTrim, 1024>(c, a, st, g);
    return q1_group_kernel<LT, DEC, kRLRep, 1024, 1024>(c, a, st, g);
}

// Shape 23: rows of > 20480 vectors in kg = ceil(vectors / 20480) segments of one
// 8-wave block each (k_q1_stats_wide's GROUP form); false when the row would need
// more segments than an XCD's CUs.
static bool q1_wide_group(lac_ctx *c, int64_t nvec, Q1Group *g) {
    const int64_t ngrp = (nvec + 63) / 64, spx = c->cus / 8;
    for (int k = (int)((nvec + kQ1WideMaxVec - 1) / kQ1WideMaxVec); k <= kQ1MaxSeg && k <= spx; k++) {
        const int64_t sp = 64 * ((ngrp + k - 1) / k), last = nvec - (k - 1) * sp;
        if (k >= 2 && last > 0 && sp <= kQ1WideMaxVec && last <= kQ1WideMaxVec) {
            g->k = k;
            g->split = (int)sp;
            g->nrb = 1;
            return true;
        }
    }
    return false;
}

template <typename LT, bool DEC>
static int q1_wide_group_kernel(lac_ctx *c, const Q1Args &a, hipStream_t st, const Q1Group &g) {
    const int64_t nvec = c->V / LogitN<LT>::N;
    if (!c->pxch) HIPCHK(hipMalloc(&c->pxch, sizeof(uint64_t) * (8 * (int64_t)c->cus + 1)));
    // rpx rows per XCD per round on rpx * k blocks of the XCD (one per CU: every member resident)
    const int64_t spx = (int64_t)(c->cus / 8), rcap = spx / g.k, rneed = (a.rows + 7) / 8;
    const int64_t rpx = rneed < rcap ? rneed : rcap;
    const unsigned grid = (unsigned)(8 * rpx * g.k);
    HIPCHK(hipMemsetAsync(c->pxch, 0, sizeof(uint64_t) * (2 * (int64_t)grid + 1), st));
    if (DEC) HIPCHK(hipMemsetAsync(c->q1chunks, 0, sizeof(uint64_t) * 64 * a.rows, st));
    else HIPCHK(hipMemsetAsync(c->stats, 0, sizeof(RowStats) * a.rows, st));
    {
        ProfScope ps(c, KID_Q1_STATS, st);
        k_q1_stats_wide<LT, kQ1WideR, DEC, true><<<grid, 512, 0, st>>>(
            (const LT *)a.lg, a.ss, a.bs, a.sym, c->B, a.rows, c->V, a.t0, a.xsh, q1_groups_per_chunk(nvec), c->stats,
            c->q1chunks, c->q1m, c->pxch, g.split, g.k, (int)rpx);
        CHECK_LAUNCH();
    }
    // repair: the tiled two-pass shape, gated on the abort word (as q1_group_kernel)
    const uint64_t *gate = c->pxch + 2 * (int64_t)grid;
    c->xch_abort = 2 * (int64_t)grid;
    if (DEC) return q1_stats_launch<LT, 16, 16, DEC, true, false, 16>(c, a, st, gate);            // shape 10
    if (sizeof(LT) == 4) return q1_stats_launch<LT, 16, 8, DEC, true, true, 16>(c, a, st, gate);  // shape 14
    return q1_stats_launch<LT, 8, 8, DEC, true, false>(c, a, st, gate);                            // shape 8
}

// The register + LDS-slot shapes (k_q1_stats_rl), by rows per block:
//   15 = one row of <= 16384 vectors (16 table copies when <= 16064: trimmed last slot, else 8),
//   17 = four rows of <= 4096 vectors (4 waves each), 18 = two rows of <= 8192 (8 waves each).
// A trimmed last slot (whole waves only) makes room for 16 table copies where the LDS allows it.
template <typename LT, bool DEC>
static int q1_stats_rl_launch(lac_ctx *c, const Q1Args &a, hipStream_t st, int shape) {
    const int64_t nvec = c->V / LogitN<LT>::N;
    switch (shape) {
    case 15:
        if (nvec <= kRLTrimMaxVec) return q1_rl_kernel<LT, DEC, 16, kRLLastTrim, 1024>(c, a, st);
        return q1_rl_kernel<LT, DEC, kRLRep, 1024, 1024>(c, a, st);
    case 17:                                       // LDS: 4 x 31 KB of slots + 16 copies (encode) / 8 (decode)
        if (nvec <= 15 * 256 + 192) return q1_rl_kernel<LT, DEC, DEC ? 8 : 16, 192, 256>(c, a, st);
        return q1_rl_kernel<LT, DEC, kRLRep, 256, 256>(c, a, st);
    default:                                       // 18 -- LDS: 2 x 61 KB of slots + 16 copies
        if (nvec <= 15 * 512 + 320) return q1_rl_kernel<LT, DEC, 16, 320, 512>(c, a, st);
        return q1_rl_kernel<LT, DEC, kRLRep, 512, 512>(c, a, st);
    }
}

// Row-group shapes (waves per row RW, 16-B vectors per thread R, rolling
// prefetch) of k_q1_stats.  AUTO takes the first listed shape that holds the row
// in registers (measured on MI355X, c3 shape: encode bf16 (8,8,y) 0.75 ms vs
// (8,8,n) 0.79 ms; decode (8,8,n) 70 M sym/s vs 46 M for the spilling (8,8,y)),
// else tiles of (8, 8); LAC_OPT_Q1_SHAPE forces one for both directions (tuning;
// identical results).  10 = tiles of a 16-wave (16,16,n) block per CU, 14 = tiles of
// (16,8) with a rolling prefetch that walks the tiles (pass 1 up, pass 2 down, then
// the next row's first tile).
//
// Round 4 retired the shapes AUTO never reaches (5, 7, 9, 11, 12, 13, 16): each vocabulary
// range resolves to one of 1..4 / 6 (rows <= 4096 vectors), 17 / 18 (<= 8192), 15
// (<= 16384), 22 (<= 26112), 19..21 / 23 (longer) or the tiled fallbacks 8 / 10 / 14,
// and a forced retired number is refused (LAC_E_ARG) instead of running a form no
// default configuration exercises.  Their measurements stay in DESIGN.md section 5b.
static const int kQ1Shapes[][3] = {{1, 4, 0}, {2, 8, 0}, {4, 8, 0}, {8, 8, 0}, {8, 16, 0}, {8, 8, 1}, {8, 4, 1}};
static bool q1_shape_live(int sh) {
    return sh >= 0 && sh <= 23 && sh != 5 && sh != 7 && sh != 9 && sh != 11 && sh != 12 && sh != 13 && sh != 16;
}

template <typename LT, bool DEC>
static int q1_stats(lac_ctx *c, const Q1Args &a, hipStream_t st) {
    const int64_t nvec = c->V / LogitN<LT>::N;
    int sh = c->q1_shape;
    auto holds = [&](int i) { return nvec <= 64 * kQ1Shapes[i - 1][0] * kQ1Shapes[i - 1][1]; };
    if (sh == 0) {
        // both directions take the prefetching (8,8) form 6 at 2049..4096 vectors: its decode
        // form spilled around the 8-way multi-sum (4 instead, no prefetch) until round 5
        // streamed the butterfly (127 VGPRs, no spills; profiles/r05/q1dec_pf/)
        static const int enc_order[] = {1, 2, 3, 6}, dec_order[] = {1, 2, 3, 6};
        // several rows per 16-wave block in registers + LDS slots (shapes 17 / 18; same-box,
        // profiles/r02/q1_rl_rows/): rows of 4097..8192 vectors in both directions (bf16
        // V = 65536 encode 1.48 -> 1.31 ms, f32 c3 1.241 -> 1.200 ms = 87 % of peak, decode
        // stats 2-3 % faster), f32 rows of 2049..4096 vectors in encode (V = 16384: 0.678 ->
        // 0.621 ms).  bf16 c3 keeps shape 6 to encode (0.651 vs 0.660 ms) and 4 to decode.
        if (nvec > 4096 && nvec <= 8192) sh = 18;
        else if (!DEC && sizeof(LT) == 4 && nvec > 2048 && nvec <= 4096) sh = 17;
        for (int i : DEC ? dec_order : enc_order) {
            if (sh) break;
            if (holds(i)) { sh = i; break; }
        }
        // rows of 8193..16384 vectors: registers + LDS slots (shape 15; same-box, bf16
        // V = 128256 encode 3.23 -> 2.49 ms = 84 % of peak, f32 V = 65536 encode 2.73 ->
        // 2.43 ms, decode 21.5 -> 24.0 M sym/s, profiles/r02/q1_rl/; bf16 decode, once its
        // spills were removed (streamed butterfly, per-group LDS totals, fresh lane index),
        // 220 -> 210 us per step of 4096 rows vs shape 9, profiles/r02/q1_rl_dec/)
        if (sh == 0 && nvec <= 16384) sh = 15;
        // rows of 16385..20480 vectors: one row per CU in the registers of an 8-wave
        // block with a rolling prefetch (shape 22; same-box vs row groups,
        // profiles/r03/wide/prefetch/: bf16 V = 151936 (Qwen2) 70.8 -> 85.6 % of peak,
        // decode stats 270 -> 184-216 us per step; bf16 131080 63 -> 73 %; f32 65540
        // 71.7 -> 80.5 %)
        // Rows of 20481..26112 vectors add 11 vectors per thread in LDS slots (same box,
        // profiles/r03/vocabs/: bf16 V = 202048 (Llama-4) 66.9 -> 81.1 %, bf16 200024
        // (o200k) 65.8 -> 76.0 %, f32 100280 (cl100k) 72.4 -> 80.4 %, f32 102400
        // (DeepSeek) 78.5 -> 86.7 %; f32 decode stats 8-11 % faster).  The bf16 decode form
        // spilled 21 VGPRs there until round 4 (hoisted LDS-DMA offsets and per-batch bin
        // addresses, now recomputed where used): spill-free, bf16 V = 202048 decode stats
        // 313 -> 269 us per step (65.9 -> 76.9 % of peak), 200024 317 -> 275 us
        // (profiles/r04/ab_dec/), so AUTO takes it in both directions
        if (sh == 0 && nvec <= kQ1WideSlotMaxVec) sh = 22;
        // longer rows: row groups (shapes 19 / 20 / 21: segments in row slots of 1 / 2 / 4
        // rows per block), the form that keeps the most bytes in flight (q1_group).
        // Round 2 had whole blocks per segment (kg = 2..4 blocks of 1 or 2 rows): bf16
        // V = 256000 48 -> 78 % of peak (profiles/r02/q1_pair_bf16/), Qwen2 bf16 57 -> 65 %
        // (profiles/r02/q1_groups2/); row slots at any kg: profiles/r03/q1_slots/
        Q1Group grp;
        if (sh == 0 && nvec > 16384 && q1_group(c, nvec, DEC, sizeof(LT) == 2, 0, &grp)) {
            // where the best slot form has several rows per block, rows go to groups of
            // 8-wave blocks instead (shape 23; same box, profiles/r03/wide/group/: bf16
            // V = 262144 68.6 -> 80.1 % of peak (slots of the 4-row form before), f32
            // 151936 79.6 -> 85.2 % (2-row form); one-row forms stay: bf16 256000 79.3 vs
            // 77.8 %, f32 128256 83.7 vs 82.5 %, f32 262144 82.2 vs 82.1 %)
            // ... and only where those blocks are well filled: segments of ~12500 vectors
            // (f32 V = 100280 / 102400, bf16 200024 / 202048: 61-63 % of a block) ran at
            // 58-70 % against 66-79 % in the slot forms (profiles/r03/vocabs/)
            Q1Group wg;
            if (grp.nrb > 1 && q1_wide_group(c, nvec, &wg) && nvec >= 0.75 * wg.k * kQ1WideMaxVec)
                return q1_wide_group_kernel<LT, DEC>(c, a, st, wg);
            return q1_stats_group_launch<LT, DEC>(c, a, st, grp);
        }
        // measured at V = 128256 f32: encode tiles of (16,8) with the tile-rolling
        // prefetch 1.98 ms vs 2.18 for tiles of (8,8) (shape 13, its (8,8) form: 2.20)
        // (rows of > 16384 vectors that no group form takes)
        if (sh == 0) sh = DEC ? 10 : (sizeof(LT) == 4 ? 14 : 8);
    }
    if (sh == 10) return q1_stats_launch<LT, 16, 16, DEC, true, false, 16>(c, a, st);   // tiles of 16384
    // registers + LDS slots (q1_stats_rl_launch): 15 one row of <= 16384 vectors per
    // block, 17 four rows of <= 4096, 18 two rows of <= 8192
    if (sh == 15 && nvec <= 16384) return q1_stats_rl_launch<LT, DEC>(c, a, st, sh);
    if (sh == 17 && nvec <= 4096) return q1_stats_rl_launch<LT, DEC>(c, a, st, 17);
    if (sh == 18 && nvec <= 8192) return q1_stats_rl_launch<LT, DEC>(c, a, st, 18);
    Q1Group grp;
    if (sh >= 19 && sh <= 21 && q1_group(c, nvec, DEC, sizeof(LT) == 2, sh == 19 ? 1 : sh == 20 ? 2 : 4, &grp))
        return q1_stats_group_launch<LT, DEC>(c, a, st, grp);
    if (sh == 22 && nvec <= kQ1WideSlotMaxVec) return q1_wide_launch<LT, DEC>(c, a, st);
    if (sh == 23 && q1_wide_group(c, nvec, &grp)) return q1_wide_group_kernel<LT, DEC>(c, a, st, grp);
    if (sh == 14) return q1_stats_launch<LT, 16, 8, DEC, true, true, 16>(c, a, st);    // tiles of (16,8,y)
    if (sh == 8) return q1_stats_launch<LT, 8, 8, DEC, true, false>(c, a, st);      // tiles of 4096 vectors
    // shapes 15, 17..23 with a row too long for them, and 1..4 / 6 likewise (kQ1Shapes
    // describes 1..7 only; lac_set_option refuses the retired shapes)
    if (sh > 7 || !q1_shape_live(sh) || !holds(sh))
        return fail(LAC_E_ARG, "q1 shape %d does not hold a row of %lld vectors", sh, (long long)nvec);
    switch (sh) {
    case 1: return q1_stats_launch<LT, 1, 4, DEC, false, false>(c, a, st);
    case 2: return q1_stats_launch<LT, 2, 8, DEC, false, false>(c, a, st);
    case 3: return q1_stats_launch<LT, 4, 8, DEC, false, false>(c, a, st);
    case 4: return q1_stats_launch<LT, 8, 8, DEC, false, false>(c, a, st);
    default: return q1_stats_launch<LT, 8, 8, DEC, false, true>(c, a, st);   // 6
    }
}

template <typename LT>
static int q1_encode(lac_ctx *c, const Q1Args &a0, int64_t steps, uint64_t *trace, hipStream_t st, int flags) {
    const unsigned blocks = (unsigned)((c->B + kWavesPerBlock - 1) / kWavesPerBlock);
    if (flags & kReset) {
        k_enc_reset<<<(unsigned)((c->B + 255) / 256), 256, 0, st>>>(c->enc, c->B, c->prec);
        CHECK_LAUNCH();
    }
    for (int64_t t0 = 0; t0 < steps; t0 += c->chunk_steps) {
        const int64_t n = (steps - t0) < c->chunk_steps ? (steps - t0) : c->chunk_steps;
        Q1Args a = a0;
        a.rows = n * c->B;
        a.t0 = t0;
        int rc = q1_stats<LT, false>(c, a, st);
        if (rc) return rc;
        {
            ProfScope ps(c, KID_ENCODE, st);
            k_encode<uint32_t><<<blocks, 64 * kWavesPerBlock, 0, st>>>(
                c->stats, a.sym, c->B, t0, n, (const uint32_t *)nullptr, 0, 0, c->V, c->prec, c->enc, c->planeA,
                c->planeC, c->cap_words, trace, LAC_MAP_CEIL, false);
        }
        CHECK_LAUNCH();
    }
    if (flags & kFinish) {
        ProfScope ps(c, KID_FINISH, st);
        k_finish<<<(unsigned)((c->B + 255) / 256), 256, 0, st>>>(c->enc, c->planeA, c->planeC, c->cap_words, c->B,
                                                                 c->prec, c->nbits, LAC_TERM_FLUSH);
        CHECK_LAUNCH();
    }
    return LAC_OK;
}

template <typename LT>
static int q1_decode(lac_ctx *c, const Q1Args &a0, int64_t steps, int32_t *out, hipStream_t st) {
    int rc0 = ensure_chunk_buffers(c);
    if (rc0) return rc0;
    const unsigned blocks = (unsigned)((c->B + kWavesPerBlock - 1) / kWavesPerBlock);
    const int64_t nvec = c->V / LogitN<LT>::N;
    for (int64_t t0 = 0; t0 < steps; t0 += c->chunk_steps) {
        const int64_t n = (steps - t0) < c->chunk_steps ? (steps - t0) : c->chunk_steps;
        Q1Args a = a0;
        a.rows = n * c->B;
        a.t0 = t0;
        int rc = q1_stats<LT, true>(c, a, st);
        if (rc) return rc;
        ProfScope ps(c, KID_Q1_DECODE, st);
        const int64_t G = q1_groups_per_chunk(nvec);
#define LAC_Q1_DEC(GC)                                                                                            \
    k_q1_decode<LT, GC><<<blocks, 64 * kWavesPerBlock, 0, st>>>((const LT *)a.lg, a.ss, a.bs, t0, n, c->V, c->prec, \
                                                               a.xsh, G, c->q1chunks, c->q1m, c->dec, c->dbits,    \
                                                               c->dstride, c->dnbits, out, c->B)
        // prec > 50 (quotients past div_small's range): the general form, 128-bit divisions
        if (c->prec > 50)
            k_q1_decode<LT, 0, false><<<blocks, 64 * kWavesPerBlock, 0, st>>>(
                (const LT *)a.lg, a.ss, a.bs, t0, n, c->V, c->prec, a.xsh, G, c->q1chunks, c->q1m, c->dec, c->dbits,
                c->dstride, c->dnbits, out, c->B);
        else switch (G) {
        case 1: LAC_Q1_DEC(1); break;
        case 2: LAC_Q1_DEC(2); break;
        case 3: LAC_Q1_DEC(3); break;
        case 4: LAC_Q1_DEC(4); break;
        case 5: LAC_Q1_DEC(5); break;
        case 6: LAC_Q1_DEC(6); break;
        case 7: LAC_Q1_DEC(7); break;
        case 8: LAC_Q1_DEC(8); break;
        default: LAC_Q1_DEC(0); break;
        }
#undef LAC_Q1_DEC
        CHECK_LAUNCH();
    }
    return LAC_OK;
}

extern "C" {

const char *lac_version(void) { return LAC_VERSION; }
const char *lac_last_error(void) { return g_err.c_str(); }

int lac_open(int device, int prec, int64_t vocab, int64_t streams, int pmf_bits, uint64_t capacity_bits,
             lac_ctx **out) {
    if (!out) return fail(LAC_E_ARG, "out is NULL");
    *out = nullptr;
    if (prec < 2 || prec > 61) return fail(LAC_E_PREC, "prec %d outside [2, 61]", prec);
    if (vocab < 1 || vocab > (int64_t)1 << 31) return fail(LAC_E_ARG, "vocab %lld outside [1, 2^31]", (long long)vocab);
    if (((int64_t)1 << (prec - 1)) < vocab)
        return fail(LAC_E_PREC, "2^(prec-1) = %lld < vocab %lld (the reference coder cannot progress)",
                    (long long)1 << (prec - 1), (long long)vocab);
    if (streams < 1) return fail(LAC_E_ARG, "streams must be >= 1");
    if (pmf_bits != 32 && pmf_bits != 64) return fail(LAC_E_ARG, "pmf_bits must be 32 or 64");
    if (capacity_bits < 64) capacity_bits = 64;
    HIPCHK(hipSetDevice(device));
    lac_ctx *c = new lac_ctx;
    c->device = device;
    if (hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || c->cus < 1)
        c->cus = 256;
    c->block_window_hi = c->cus;                      // 256 on MI355X
    c->block_window_lo = (c->cus * 5) / 8;            // 160 on MI355X (measured, profiles/r01/decode_paths_v2/)
    c->prec = prec;
    c->pmf_bits = pmf_bits;
    c->V = vocab;
    c->B = streams;
    c->cap_bits = capacity_bits;
    c->cap_words = (capacity_bits + 63) / 64 + 1;
    hipError_t e = hipSuccess;
    // split path: steps per row-stats launch, enough rows to fill the chip even for 1 stream
    c->chunk_steps = streams >= 512 ? kChunkSteps : ((32768 / streams + 63) / 64) * 64;
    e = e ? e : hipMalloc(&c->stats, sizeof(RowStats) * c->chunk_steps * streams);
    e = e ? e : hipMalloc(&c->enc, sizeof(EncState) * streams);
    e = e ? e : hipMalloc(&c->dec, sizeof(DecState) * streams);
    e = e ? e : hipMalloc(&c->planeA, sizeof(uint64_t) * (c->cap_words * streams + 1));
    e = e ? e : hipMalloc(&c->planeC, sizeof(uint64_t) * (c->cap_words * streams + 1));
    e = e ? e : hipMalloc(&c->nbits, sizeof(uint64_t) * streams);
    e = e ? e : hipMemset(c->nbits, 0, sizeof(uint64_t) * streams);
    c->own_planeA = c->planeA;
    c->own_nbits = c->nbits;
    if (e != hipSuccess) {
        lac_close(c);
        return fail(LAC_E_HIP, "device allocation: %s", hipGetErrorString(e));
    }
    int rc = lac_encode_reset(c, nullptr);
    if (rc) { lac_close(c); return rc; }
    if ((e = hipDeviceSynchronize()) != hipSuccess) {
        lac_close(c);
        return fail(LAC_E_HIP, "hipDeviceSynchronize: %s", hipGetErrorString(e));
    }
    *out = c;
    return LAC_OK;
}

int lac_close(lac_ctx *c) {
    if (!c) return LAC_OK;
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    (void)hipFree(c->stats);
    (void)hipFree(c->enc);
    (void)hipFree(c->dec);
    (void)hipFree(c->tail);
    (void)hipFree(c->own_planeA ? c->own_planeA : c->planeA);
    (void)hipFree(c->planeC);
    (void)hipFree(c->own_nbits ? c->own_nbits : c->nbits);
    (void)hipFree(c->q1chunks);
    (void)hipFree(c->dmeta);
    (void)hipFree(c->dresume);
    (void)hipFree(c->lvpre);
    (void)hipFree(c->lchunk);
    (void)hipFree(c->lmeta);
    (void)hipFree(c->dprogress);
    (void)hipFree(c->q1m);
    (void)hipFree(c->pxch);
    for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
    delete c;
    return LAC_OK;
}

int lac_encode_reset(lac_ctx *c, void *stream) {
    if (!c) return fail(LAC_E_ARG, "ctx is NULL");
    HIPCHK(hipSetDevice(c->device));
    c->mode = 0;
    c->finished = 0;
    k_enc_reset<<<(unsigned)((c->B + 255) / 256), 256, 0, S(stream)>>>(c->enc, c->B, c->prec);
    CHECK_LAUNCH();
    return LAC_OK;
}

int lac_encode_rebase(lac_ctx *c, void *stream) {
    if (!c) return fail(LAC_E_ARG, "ctx is NULL");
    if (c->mode != 0) return fail(LAC_E_STATE, "context is decoding");
    HIPCHK(hipSetDevice(c->device));
    k_enc_rebase<<<(unsigned)((c->B + 255) / 256), 256, 0, S(stream)>>>(c->enc, c->B);
    CHECK_LAUNCH();
    return LAC_OK;
}

int lac_encode(lac_ctx *c, const void *pmf_dev, int64_t step_stride, int64_t stream_stride, const int32_t *sym_dev,
               int64_t steps, uint64_t *trace_dev, void *stream) {
    if (c && c->mode != 0) return fail(LAC_E_STATE, "context is decoding; call lac_encode_reset first");
    const int rc = encode_dispatch(c, pmf_dev, step_stride, stream_stride, sym_dev, steps, trace_dev, stream, 0);
    if (rc == LAC_OK && steps > 0) c->finished = 0;
    return rc;
}

int lac_encode_job(lac_ctx *c, const void *pmf_dev, int64_t step_stride, int64_t stream_stride,
                   const int32_t *sym_dev, int64_t steps, uint64_t *trace_dev, void *stream) {
    const int rc = encode_dispatch(c, pmf_dev, step_stride, stream_stride, sym_dev, steps, trace_dev, stream,
                                   kReset | kFinish);
    if (rc == LAC_OK) c->finished = 1;
    return rc;
}

int lac_set_option(lac_ctx *c, int option, int64_t value) {
    if (!c) return fail(LAC_E_ARG, "ctx is NULL");
    switch (option) {
    case LAC_OPT_ENCODE_PATH:
        if (value < LAC_PATH_AUTO || value > LAC_PATH_FUSED) return fail(LAC_E_ARG, "bad encode path %lld", (long long)value);
        c->path = (int)value;
        return LAC_OK;
    case LAC_OPT_FUSED_MIN_STREAMS:
        if (value < 1) return fail(LAC_E_ARG, "fused_min_streams must be >= 1");
        c->fused_min_streams = value;
        return LAC_OK;
    case LAC_OPT_DECODE_PATH:
        if (value < LAC_PATH_AUTO || value > LAC_PATH_BLOCK) return fail(LAC_E_ARG, "bad decode path");
        c->dpath = (int)value;
        return LAC_OK;
    case LAC_OPT_BLOCK_WAVES:
        if (value != 0 && value != 4 && value != 8 && value != 16) return fail(LAC_E_ARG, "block waves: 0, 4, 8 or 16");
        c->block_waves = (int)value;
        return LAC_OK;
    case LAC_OPT_DECODE_FINE:
        if (value != 0 && value != 1) return fail(LAC_E_ARG, "decode_fine must be 0 or 1");
        c->fine_decode = (int)value;
        return LAC_OK;
    case LAC_OPT_Q1_SHAPE:
        if (!q1_shape_live((int)value) || value != (int)value) return fail(LAC_E_ARG, "bad or retired q1 shape");
        c->q1_shape = (int)value;
        return LAC_OK;
    case LAC_OPT_MAPPING:
        if (value != LAC_MAP_CEIL && value != LAC_MAP_FLOOR) return fail(LAC_E_ARG, "bad mapping");
        c->mapping = (int)value;
        return LAC_OK;
    case LAC_OPT_TERMINATION:
        if (value != LAC_TERM_FLUSH && value != LAC_TERM_ACSAMPLER) return fail(LAC_E_ARG, "bad termination");
        c->term = (int)value;
        return LAC_OK;
    default:
        return fail(LAC_E_ARG, "unknown option %d", option);
    }
}

int lac_encode_finish(lac_ctx *c, void *stream) {
    if (!c) return fail(LAC_E_ARG, "ctx is NULL");
    if (c->mode != 0) return fail(LAC_E_STATE, "context is decoding");
    HIPCHK(hipSetDevice(c->device));
    ProfScope ps(c, KID_FINISH, S(stream));
    c->finished = 1;
    k_finish<<<(unsigned)((c->B + 255) / 256), 256, 0, S(stream)>>>(c->enc, c->planeA, c->planeC, c->cap_words, c->B,
                                                                   c->prec, c->nbits, c->term);
    CHECK_LAUNCH();
    return LAC_OK;
}

int lac_stream_status(lac_ctx *c, int32_t *err_host, int64_t *err_step_host, void *stream) {
    if (!c) return fail(LAC_E_ARG, "ctx is NULL");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(S(stream)));
    int first = LAC_OK;
    if (c->mode == 0) {
        std::vector<EncState> v(c->B);
        HIPCHK(hipMemcpy(v.data(), c->enc, sizeof(EncState) * c->B, hipMemcpyDeviceToHost));
        for (int64_t b = 0; b < c->B; b++) {
            if (err_host) err_host[b] = v[b].err;
            if (err_step_host) err_step_host[b] = v[b].err ? v[b].err_step : -1;
            if (!first && v[b].err) first = v[b].err;
        }
    } else {
        std::vector<DecState> v(c->B);
        HIPCHK(hipMemcpy(v.data(), c->dec, sizeof(DecState) * c->B, hipMemcpyDeviceToHost));
        for (int64_t b = 0; b < c->B; b++) {
            if (err_host) err_host[b] = v[b].err;
            if (err_step_host) err_step_host[b] = v[b].err ? v[b].err_step : -1;
            if (!first && v[b].err) first = v[b].err;
        }
    }
    if (first) fail(first, "a stream reported status %d", first);
    return first;
}

int lac_encoded_lengths(lac_ctx *c, uint64_t *nbits_host, void *stream) {
    if (!c || !nbits_host) return fail(LAC_E_ARG, "NULL argument");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(S(stream)));
    HIPCHK(hipMemcpy(nbits_host, c->nbits, sizeof(uint64_t) * c->B, hipMemcpyDeviceToHost));
    return LAC_OK;
}

int lac_encoded_device(lac_ctx *c, const uint8_t **bits_dev, uint64_t *stride_bytes, const uint64_t **nbits_dev) {
    if (!c) return fail(LAC_E_ARG, "ctx is NULL");
    if (bits_dev) *bits_dev = reinterpret_cast<const uint8_t *>(c->planeA);
    if (stride_bytes) *stride_bytes = c->cap_words * 8;
    if (nbits_dev) *nbits_dev = c->nbits;
    return LAC_OK;
}

int lac_copy_bits(lac_ctx *c, uint8_t *dst, uint64_t dst_stride, void *stream) {
    if (!c || !dst || dst_stride == 0) return fail(LAC_E_ARG, "bad argument");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(S(stream)));
    const uint64_t src_stride = c->cap_words * 8;
    const uint64_t width = dst_stride < src_stride ? dst_stride : src_stride;
    HIPCHK(hipMemcpy2D(dst, dst_stride, c->planeA, src_stride, width, (size_t)c->B, hipMemcpyDeviceToHost));
    return LAC_OK;
}

int lac_copy_bits_dev(lac_ctx *c, uint8_t *dst, uint64_t dst_stride, void *stream) {
    if (!c || !dst || dst_stride == 0) return fail(LAC_E_ARG, "bad argument");
    HIPCHK(hipSetDevice(c->device));
    const uint64_t src_stride = c->cap_words * 8;
    const uint64_t width = dst_stride < src_stride ? dst_stride : src_stride;
    HIPCHK(hipMemcpy2DAsync(dst, dst_stride, c->planeA, src_stride, width, (size_t)c->B, hipMemcpyDeviceToDevice,
                            S(stream)));
    return LAC_OK;
}

int lac_pack_jobs(int device, const uint64_t *planeA_dev, uint64_t plane_stride, const uint64_t *nbits_dev,
                  int64_t jobs, int64_t streams, uint64_t cap_words, uint8_t *dst, uint64_t dst_bytes, int hdr_bytes,
                  const uint64_t *base_dev, uint64_t *ends_dev, uint64_t *lens_out, void *stream) {
    if (!dst || !ends_dev || streams < 0 || jobs < 1 || jobs > 65535 ||
        (streams > 0 && (!planeA_dev || !nbits_dev)) || (hdr_bytes != 2 && hdr_bytes != 4) ||
        (jobs > 1 && plane_stride < (uint64_t)streams * cap_words))
        return fail(LAC_E_ARG, "bad argument");
    if (hdr_bytes == 2 && cap_words * 64 >= 65536)
        return fail(LAC_E_ARG, "a 2-byte header holds bit counts below 65536; these streams hold up to "
                               "%llu bits: use 4", (unsigned long long)(cap_words * 64));
    HIPCHK(hipSetDevice(device));
    const unsigned bx = (unsigned)((streams + 1023) / 1024);
    k_pack<<<dim3(bx > 0 ? bx : 1, (unsigned)jobs), 1024, 0, S(stream)>>>(
        planeA_dev, plane_stride, cap_words, nbits_dev, streams, hdr_bytes, dst, dst_bytes, base_dev, ends_dev,
        lens_out);
    CHECK_LAUNCH();
    return LAC_OK;
}

int lac_pack_bits_at(lac_ctx *c, uint8_t *dst, uint64_t dst_bytes, int hdr_bytes, const uint64_t *base_dev,
                     uint64_t *end_dev, uint64_t *len_out, void *stream) {
    if (!c) return fail(LAC_E_ARG, "ctx is NULL");
    if (c->mode != 0) return fail(LAC_E_STATE, "context is decoding");
    if (!c->finished) return fail(LAC_E_STATE, "no finished encode to pack (lac_encode_job or lac_encode_finish)");
    return lac_pack_jobs(c->device, c->planeA, 0, c->nbits, 1, c->B, c->cap_words, dst, dst_bytes, hdr_bytes,
                         base_dev, end_dev, len_out, stream);
}

int lac_set_output(lac_ctx *c, uint64_t *planeA_dev, uint64_t *nbits_dev) {
    if (!c) return fail(LAC_E_ARG, "ctx is NULL");
    if (!planeA_dev != !nbits_dev) return fail(LAC_E_ARG, "planeA_dev and nbits_dev: both or neither");
    if ((uintptr_t)planeA_dev % 8 || (uintptr_t)nbits_dev % 8) return fail(LAC_E_ARG, "buffers must be 8-byte aligned");
    c->planeA = planeA_dev ? planeA_dev : c->own_planeA;
    c->nbits = nbits_dev ? nbits_dev : c->own_nbits;
    c->finished = 0;
    return LAC_OK;
}

int lac_pack_bits(lac_ctx *c, uint8_t *dst, int hdr_bytes, uint64_t *len_dev, void *stream) {
    if (!len_dev) return fail(LAC_E_ARG, "bad argument");
    return lac_pack_bits_at(c, dst, ~0ull, hdr_bytes, nullptr, len_dev, nullptr, stream);
}

int lac_host_alloc(uint64_t bytes, void **host_out, void **dev_out) {
    if (!host_out || !dev_out || bytes == 0) return fail(LAC_E_ARG, "bad argument");
    void *h = nullptr;
    HIPCHK(hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocCoherent));
    void *d = nullptr;
    const hipError_t e = hipHostGetDevicePointer(&d, h, 0);
    if (e != hipSuccess) {
        (void)hipHostFree(h);
        return fail(LAC_E_HIP, "hipHostGetDevicePointer: %s", hipGetErrorString(e));
    }
    memset(h, 0, bytes);
    *host_out = h;
    *dev_out = d;
    return LAC_OK;
}

int lac_host_free(void *host) {
    if (host) HIPCHK(hipHostFree(host));
    return LAC_OK;
}

int lac_copy_nbits_dev(lac_ctx *c, uint64_t *dst, void *stream) {
    if (!c || !dst) return fail(LAC_E_ARG, "bad argument");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpyAsync(dst, c->nbits, sizeof(uint64_t) * c->B, hipMemcpyDeviceToDevice, S(stream)));
    return LAC_OK;
}

int lac_encoder_registers(lac_ctx *c, int64_t *l_host, int64_t *h_host, void *stream) {
    if (!c) return fail(LAC_E_ARG, "ctx is NULL");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(S(stream)));
    std::vector<EncState> v(c->B);
    HIPCHK(hipMemcpy(v.data(), c->enc, sizeof(EncState) * c->B, hipMemcpyDeviceToHost));
    for (int64_t b = 0; b < c->B; b++) {
        if (l_host) l_host[b] = v[b].l;
        if (h_host) h_host[b] = v[b].h;
    }
    return LAC_OK;
}

static_assert(sizeof(lac_enc_state) == sizeof(EncState) && offsetof(lac_enc_state, nflush) == offsetof(EncState, nflush) &&
                  offsetof(lac_enc_state, flush) == offsetof(EncState, flush),
              "lac_enc_state mirrors EncState");

int lac_encode_get_state(lac_ctx *c, lac_enc_state *host_out, uint64_t *planes_host, void *stream) {
    if (!c || !host_out) return fail(LAC_E_ARG, "NULL argument");
    if (c->mode != 0) return fail(LAC_E_STATE, "context is decoding");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpyAsync(host_out, c->enc, sizeof(EncState) * c->B, hipMemcpyDeviceToHost, S(stream)));
    if (planes_host) {
        const size_t n = sizeof(uint64_t) * c->cap_words * c->B;
        HIPCHK(hipMemcpyAsync(planes_host, c->planeA, n, hipMemcpyDeviceToHost, S(stream)));
        HIPCHK(hipMemcpyAsync(planes_host + c->cap_words * c->B, c->planeC, n, hipMemcpyDeviceToHost, S(stream)));
    }
    HIPCHK(hipStreamSynchronize(S(stream)));
    return LAC_OK;
}

int lac_encode_set_state(lac_ctx *c, const lac_enc_state *host_in, const uint64_t *planes_host, void *stream) {
    if (!c || !host_in) return fail(LAC_E_ARG, "NULL argument");
    if (c->mode != 0) return fail(LAC_E_STATE, "context is decoding; call lac_encode_reset first");
    const int64_t D = (int64_t)1 << c->prec;
    for (int64_t b = 0; b < c->B; b++) {
        const lac_enc_state &q = host_in[b];
        if (q.err) continue;
        if (q.L > 0 && !planes_host)
            return fail(LAC_E_ARG, "stream %lld has %lld bits written: its planes must be restored too",
                        (long long)b, (long long)q.L);
        if (q.l < 0 || q.l >= 2 * D || q.h < q.l || q.h - q.l >= D || q.L > c->cap_words * 64 || q.nsym < 0 ||
            q.nflush < -1 || q.nflush > 8)
            return fail(LAC_E_ARG, "stream %lld: encoder registers out of range", (long long)b);
    }
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpyAsync(c->enc, host_in, sizeof(EncState) * c->B, hipMemcpyHostToDevice, S(stream)));
    if (planes_host) {
        const size_t n = sizeof(uint64_t) * c->cap_words * c->B;
        HIPCHK(hipMemcpyAsync(c->planeA, planes_host, n, hipMemcpyHostToDevice, S(stream)));
        HIPCHK(hipMemcpyAsync(c->planeC, planes_host + c->cap_words * c->B, n, hipMemcpyHostToDevice, S(stream)));
    }
    c->finished = 0;
    HIPCHK(hipStreamSynchronize(S(stream)));
    return LAC_OK;
}

int lac_flush_digits(lac_ctx *c, int8_t *digits_host, int32_t *count_host, void *stream) {
    if (!c) return fail(LAC_E_ARG, "ctx is NULL");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(S(stream)));
    std::vector<EncState> v(c->B);
    HIPCHK(hipMemcpy(v.data(), c->enc, sizeof(EncState) * c->B, hipMemcpyDeviceToHost));
    for (int64_t b = 0; b < c->B; b++) {
        if (count_host) count_host[b] = v[b].nflush;
        if (digits_host) memcpy(digits_host + 8 * b, v[b].flush, 8);
    }
    return LAC_OK;
}

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

static int logits_encode(lac_ctx *c, const void *logits_dev, int logit_type, int64_t step_stride,
                         int64_t stream_stride, const int32_t *sym_dev, int64_t steps, uint64_t *trace_dev,
                         void *stream, int flags) {
    if (!c || (steps > 0 && (!logits_dev || !sym_dev))) return fail(LAC_E_ARG, "NULL argument");
    int rc = logits_check(c, logits_dev, logit_type, step_stride, stream_stride, steps);
    uint32_t xsh = 0;
    if (rc || (rc = q1_shift(c, &xsh))) return rc;
    if (steps == 0 && !flags) return LAC_OK;
    HIPCHK(hipSetDevice(c->device));
    c->mode = 0;
    const Q1Args a{logits_dev, step_stride, stream_stride, sym_dev, 0, 0, xsh};
    return logit_type == LAC_LOGITS_BF16 ? q1_encode<uint16_t>(c, a, steps, trace_dev, S(stream), flags)
                                         : q1_encode<float>(c, a, steps, trace_dev, S(stream), flags);
}

int lac_encode_logits_job(lac_ctx *c, const void *logits_dev, int logit_type, int64_t step_stride,
                          int64_t stream_stride, const int32_t *sym_dev, int64_t steps, uint64_t *trace_dev,
                          void *stream) {
    const int rc = logits_encode(c, logits_dev, logit_type, step_stride, stream_stride, sym_dev, steps, trace_dev,
                                 stream, kReset | kFinish);
    if (rc == LAC_OK) c->finished = 1;
    return rc;
}

int lac_encode_logits(lac_ctx *c, const void *logits_dev, int logit_type, int64_t step_stride,
                      int64_t stream_stride, const int32_t *sym_dev, int64_t steps, uint64_t *trace_dev,
                      void *stream) {
    const int rc = logits_encode(c, logits_dev, logit_type, step_stride, stream_stride, sym_dev, steps, trace_dev,
                                 stream, 0);
    if (rc == LAC_OK && steps > 0) c->finished = 0;
    return rc;
}

int lac_decode_logits_steps(lac_ctx *c, const void *logits_dev, int logit_type, int64_t step_stride,
                            int64_t stream_stride, int64_t steps, int32_t *sym_out_dev, void *stream) {
    if (!c || (steps > 0 && (!logits_dev || !sym_out_dev))) return fail(LAC_E_ARG, "NULL argument");
    if (c->mode != 1) return fail(LAC_E_STATE, "call lac_decode_open first");
    int rc = logits_check(c, logits_dev, logit_type, step_stride, stream_stride, steps);
    uint32_t xsh = 0;
    if (rc || (rc = q1_shift(c, &xsh))) return rc;
    if (steps == 0) return LAC_OK;
    HIPCHK(hipSetDevice(c->device));
    const Q1Args a{logits_dev, step_stride, stream_stride, nullptr, 0, 0, xsh};
    return logit_type == LAC_LOGITS_BF16 ? q1_decode<uint16_t>(c, a, steps, sym_out_dev, S(stream))
                                         : q1_decode<float>(c, a, steps, sym_out_dev, S(stream));
}

int lac_quantize_logits(lac_ctx *c, const void *logits_dev, int logit_type, int64_t step_stride,
                        int64_t stream_stride, int64_t steps, uint32_t *pmf_out_dev, void *stream) {
    if (!c || (steps > 0 && (!logits_dev || !pmf_out_dev))) return fail(LAC_E_ARG, "NULL argument");
    if (logit_type != LAC_LOGITS_BF16 && logit_type != LAC_LOGITS_F32) return fail(LAC_E_ARG, "logit type");
    const int n = logit_type == LAC_LOGITS_BF16 ? 8 : 4;
    if (steps < 0 || step_stride < 0 || stream_stride < 0) return fail(LAC_E_ARG, "negative size/stride");
    if (steps > 0 && ((uintptr_t)logits_dev % 16 || c->V % n || step_stride % n || stream_stride % n))
        return fail(LAC_E_ARG, "logits rows must be 16-byte aligned with vocab and strides multiples of %d", n);
    uint32_t xsh = 0;
    int rc = q1_shift(c, &xsh);
    if (rc) return rc;
    if (steps == 0) return LAC_OK;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = S(stream);
    const int64_t rows = steps * c->B;
    const unsigned blocks = (unsigned)((rows + kWavesPerBlock - 1) / kWavesPerBlock);
    if (logit_type == LAC_LOGITS_BF16)
        k_quantize_logits<uint16_t><<<blocks, 64 * kWavesPerBlock, 0, st>>>(
            (const uint16_t *)logits_dev, step_stride, stream_stride, c->B, rows, c->V, xsh, pmf_out_dev);
    else
        k_quantize_logits<float><<<blocks, 64 * kWavesPerBlock, 0, st>>>(
            (const float *)logits_dev, step_stride, stream_stride, c->B, rows, c->V, xsh, pmf_out_dev);
    CHECK_LAUNCH();
    return LAC_OK;
}

int lac_q1_k(int prec, int64_t vocab) {
    int cl = 0;
    while (((int64_t)1 << cl) < vocab) cl++;
    const int k = prec - 1 - cl;
    return k > LAC_Q1_KMAX ? LAC_Q1_KMAX : k;
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

// ---- host-side register arithmetic for predictors with their own mapping --------
// (include/lac.h "predictor-mapped coding"; no device work): lac_hc.h, shared with
// the host sanitizer build (tests/native)
int lac_hc_encode_symbol(int prec, int64_t *l, int64_t *h, int64_t lo, int64_t hi, int8_t *digits,
                         int32_t *ndigits) {
    const char *msg = "";
    const int rc = lac::hc::encode_symbol(prec, l, h, lo, hi, digits, ndigits, &msg);
    return rc ? fail(rc, "%s", msg) : LAC_OK;
}

int lac_hc_encode_flush(int prec, int64_t l, int64_t h, int8_t *digits, int32_t *ndigits) {
    const char *msg = "";
    const int rc = lac::hc::encode_flush(prec, l, h, digits, ndigits, &msg);
    return rc ? fail(rc, "%s", msg) : LAC_OK;
}

int lac_hc_decode_emit(int prec, int64_t *regs, int64_t lo, int64_t hi, int renormalise) {
    const char *msg = "";
    const int rc = lac::hc::decode_emit(prec, regs, lo, hi, renormalise, &msg);
    return rc ? fail(rc, "%s", msg) : LAC_OK;
}

int lac_q1_group_aborted(lac_ctx *c, int64_t *aborted, void *stream) {
    if (!c || !aborted) return fail(LAC_E_ARG, "NULL argument");
    *aborted = 0;
    if (c->xch_abort < 0 || !c->pxch) return LAC_OK;
    HIPCHK(hipSetDevice(c->device));
    uint64_t v = 0;
    HIPCHK(hipMemcpyAsync(&v, c->pxch + c->xch_abort, sizeof v, hipMemcpyDeviceToHost, S(stream)));
    HIPCHK(hipStreamSynchronize(S(stream)));
    *aborted = v ? 1 : 0;
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

int lac_profile_enable(lac_ctx *c, int on) {
    if (!c) return fail(LAC_E_ARG, "ctx is NULL");
    c->prof = on != 0;
    return LAC_OK;
}

int lac_profile_read(lac_ctx *c, double *ms_total, int64_t *launches, int reset) {
    if (!c) return fail(LAC_E_ARG, "ctx is NULL");
    HIPCHK(hipSetDevice(c->device));
    double tot[KID_COUNT] = {0};
    int64_t cnt[KID_COUNT] = {0};
    for (auto &u : c->ev_used) {
        HIPCHK(hipEventSynchronize(u.second.second));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, u.second.first, u.second.second));
        tot[u.first] += ms;
        cnt[u.first] += 1;
    }
    for (int k = 0; k < KID_COUNT; k++) {
        if (ms_total) ms_total[k] = tot[k];
        if (launches) launches[k] = cnt[k];
    }
    if (reset) {
        c->ev_used.clear();
        c->ev_next = 0;
    }
    return LAC_OK;
}

}  // extern "C"
