// lac_logits.hip -- the fused logits path of liblac.so:
// logits rows -> q1 tables (include/lac_q1_table.h, an integer-exact restatement of
// llama_compress.py:24-30's quantiser) -> the coder, with no pmf in HBM.  k_q1_stats
// (and its register + LDS-slot and 8-wave forms k_q1_stats_rl / _wide, row groups)
// computes each row's RowStats (encode) or maximum and 64 chunk totals (decode);
// k_q1_decode is the sequential decode over them; k_quantize_logits materialises
// tables.  DESIGN.md section 5b.
#include "lac_host.h"
#include "lac_dec_dev.h"

namespace {

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
#ifndef LAC_Q1_DEC_DIRECT
#define LAC_Q1_DEC_DIRECT 1      // k_q1_stats decode form, one row per block of 64 groups: per-wave chunk stores
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
    // decode form, rows of <= 64 groups of 64 vectors owned by a whole block (shapes 4 / 6,
    // bf16 c3): each wave stores its 8 group totals -- the row's chunk totals, since G = 1
    // there -- straight to HBM, with no LDS bins, no second barrier and no writer wave;
    // the maxima's LDS words alternate between rows, so a wave may start the next row
    // while the others still read this one's
    constexpr bool DIRECT = DEC && !MULTI && RW * R == 64 && !LAC_Q1_DEFER_DEC && LAC_Q1_DEC_DIRECT;
    __shared__ float smax[2][NWB];
    __shared__ int smaxi[2][NWB];
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
    int par = 0;
    for (int64_t rb = (int64_t)blockIdx.x * NR; rb < rows; rb += stride, par ^= 1) {
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
            if (lane == 0) smaxi[par][w] = wi;
            if (!DEC && gt == 0) sps[g] = 0;
            __syncthreads();
            int bi = smaxi[par][0];
#pragma unroll
            for (int i = 1; i < NWB; i++) bi = smaxi[par][i] > bi ? smaxi[par][i] : bi;
            if (bi >= 0 && bi <= 0x7F80) {                    // block-uniform
                m = __uint_as_float((uint32_t)bi << 16);
            } else {
#pragma unroll
                for (int j = 0; j < R; j++)
#pragma unroll
                    for (int e = 0; e < N; e++) mx = fmaxf(mx, logit_at<LT>(x[j], e));
                mx = wave_max_f32(mx);
                if (lane == 0) smax[par][w] = mx;
                __syncthreads();
                m = smax[par][0];
#pragma unroll
                for (int i = 1; i < NWB; i++) m = fmaxf(m, smax[par][i]);
            }
        } else {
            mx = wave_max_f32(mx);
            if (lane == 0) smax[par][w] = mx;
            if (!DEC && gt == 0) sps[g] = 0;
            __syncthreads();
            m = smax[par][g * RW];
#pragma unroll
            for (int i = 1; i < RW; i++) m = fmaxf(m, smax[par][g * RW + i]);
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
                if constexpr (DIRECT) {                        // every chunk once: grp covers 0..63
                    const int grp = wg + RW * q_index<R>(lane);
                    if (lane < R && valid) chunks[r * 64 + grp] = grp * 64 < nvec ? gsum : 0;
                } else if (lane < R) {
                    const int grp = tile * RW * R + wg + RW * q_index<R>(lane);
                    if (grp * 64 < nvec) atomicAdd(&bins[g][grp / (int)G], (unsigned long long)gsum);
                }
            }
        }
        if (!DEC) {
            const uint64_t t64 = wave_sum_u64(tot), l64 = wave_sum_u64(lo);
            if (lane == 0) { ssum[w][0] = t64; ssum[w][1] = l64; }
        }
        if constexpr (DIRECT) {
            if (valid && w == 0 && lane == 0) mrow[r] = m;
        } else {
            __syncthreads();
        }
        if (DEC) {
            if (!DIRECT && wg == 0) {
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
                tgt = div_small_u<false>(v, T, 0, w, iw);
                thi = vh == v ? tgt : (vh < w ? div_small_u<false>(vh, T, 0, w, iw) : 0);
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
                        div_small_u2<false>(lo_c, hi_c, w, T - 1, T, recip(T), &a, &bb);
                    } else {
                        div_pair(lo_c, hi_c, w, T - 1, T, recip(T), &a, &bb);
                    }
                    const bool det = vh < w && thi < hi_c;
                    if (st.det && det) st.ndet++;
                    else st.det = 0;
                    err = LAC_Q1D_NB ? decode_advance_nb(st, a, bb, win, mynbits, prec)
                                     : decode_advance<true>(st, a, bb, win, mynbits, prec);
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


}  // namespace

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
bool q1_shape_live(int sh) {
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
    int rc;
    if ((flags & kReset) && (rc = enc_reset_launch(c, st))) return rc;
    for (int64_t t0 = 0; t0 < steps; t0 += c->chunk_steps) {
        const int64_t n = (steps - t0) < c->chunk_steps ? (steps - t0) : c->chunk_steps;
        Q1Args a = a0;
        a.rows = n * c->B;
        a.t0 = t0;
        if ((rc = q1_stats<LT, false>(c, a, st))) return rc;
        if ((rc = enc_stats_launch(c, a.sym, t0, n, trace, st))) return rc;   // k_encode over the stats
    }
    if ((flags & kFinish) && (rc = enc_finish_launch(c, LAC_TERM_FLUSH, st))) return rc;
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
    if (rc == LAC_OK) enc_mark_finished(c);
    return rc;
}

int lac_encode_logits(lac_ctx *c, const void *logits_dev, int logit_type, int64_t step_stride,
                      int64_t stream_stride, const int32_t *sym_dev, int64_t steps, uint64_t *trace_dev,
                      void *stream) {
    const int rc = logits_encode(c, logits_dev, logit_type, step_stride, stream_stride, sym_dev, steps, trace_dev,
                                 stream, 0);
    if (rc == LAC_OK && steps > 0) enc_mark_open(c);
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

}  // extern "C"
