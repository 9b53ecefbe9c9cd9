// lac_encode.hip -- the encode family of liblac.so: A_to_bin's range-update loop
// (arith_code.py:169-246) over per-token integer pmf rows.
//
//   k_row_stats   one wave per (step, stream) row.  HBM-bound scan of the integer
//                 pmf row (16-B coalesced loads, 8 in flight per lane) producing the
//                 four scalars the reference's symbol_to_range needs
//                 (arith_code.py:79-110): lo = c_{s-1}, hi = c_s, T = c_{V-1}, minp.
//   k_encode      one wave per stream, sequential over a chunk's steps: the range
//                 narrowing + renormalisation (:169-192).  Lane i prefetches step i's
//                 stats; rows that hit fudged_dist (:83-93) are re-scanned by the wave.
//   k_encode_fused  at >= 2048 streams: one launch per job, one wave per stream,
//                 row scan + coder step + reset + flush + pack in one kernel.
//   k_finish      flush (:193-202), carry resolution of bits() (:227-246), MSB-first
//                 byte packing of group_bits (:336-347), one lane per stream.
//   k_pack        the multi-GPU gather's payload (lac_pack_jobs, lac_amd/dist.py).
#include "lac_host.h"

#include <type_traits>

namespace {

#if LAC_ENC_PHASES
__device__ unsigned long long g_enc_phase[8];
#endif
constexpr int kEncUnroll = LAC_ENC_UNROLL;

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

// k_encode's straight steps over one 64-step block (see k_encode): step i's row values
// out of lane i (LAC_ENC_PIPE: read one step ahead, off the chain), the two mul-divs
// through the row fractions (T32: 32 x 64-bit remainder products), renorm() without its
// kk <= 0 branch (kk = 0 keeps l and h, e = 0), plane_append's one-word case inline.  The
// inner loop leaves only at the block's end, at a step whose digits cross a plane word
// (~1 step in 7; its append runs after the loop, which then resumes) and, FT (a row of the
// block can fudge: T > 2^(prec-1)), at a fudged step, before it changes anything; so one
// exit test per step (two with FT).  Returns the first step not done (n at the block's
// end); results, registers and error steps are coder_step's.
struct SP {
    uint64_t lo, hi, tot, flo, fhi, fthr;              // this lane's row values (lane i: step i)
    int n, prec;
    uint64_t cap_words, *pa, *pc;
    int lane;
};
template <bool CEIL, bool T32, bool FT>
__device__ inline int straight_steps(const SP &sp, EncState &st, int64_t &l, int64_t &h, bool &ok) {
    auto store = [&](uint64_t idx, uint64_t wa, uint64_t wc) {
        if (sp.lane == 0) { sp.pa[idx] = wa; sp.pc[idx] = wc; }
    };
    typedef typename std::conditional<T32, uint32_t, uint64_t>::type CT;   // counts and totals
    struct Row {
        CT lo, hi, T;
        uint64_t fl, fh, ft;
    };
    auto rd = [&](int j) {
        Row r;
        if constexpr (T32) {
            r.lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)sp.lo, j);
            r.hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)sp.hi, j);
            r.T = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)sp.tot, j);
        } else {
            r.lo = readlane_u64(sp.lo, j);
            r.hi = readlane_u64(sp.hi, j);
            r.T = readlane_u64(sp.tot, j);
        }
        r.fl = readlane_u64(sp.flo, j);
        r.fh = readlane_u64(sp.fhi, j);
        r.ft = FT ? readlane_u64(sp.fthr, j) : 0;
        return r;
    };
    const int n = sp.n, prec = sp.prec;
    const int64_t nsym0 = st.nsym;
    Row nx = rd(0);
    int i = 0;
    int kk = 0;
    uint64_t e = 0;
    bool fudged = false;
    while (i < n) {
        for (; i < n; i++) {
            const Row r = LAC_ENC_PIPE ? nx : rd(i);
            if constexpr (LAC_ENC_PIPE) nx = rd(i + 1 < n ? i + 1 : i);
            const uint64_t w = (uint64_t)(h - l + 1);
            if constexpr (FT) {
                if (!nonneg_uni((int64_t)(w - r.ft))) {         // fudged (arith_code.py:84): the general step
                    fudged = true;
                    break;
                }
            }
            uint64_t a, bb;
            if constexpr (T32) {
                a = frac_mul_div32<CEIL>(r.fl, r.lo, w, r.T);
                bb = frac_mul_div32<CEIL>(r.fh, r.hi, w, r.T);
            } else {
                a = frac_mul_div<true>(r.fl, r.lo, w, r.T, CEIL);
                bb = frac_mul_div<true>(r.fh, r.hi, w, r.T, CEIL);
            }
            h = l + (int64_t)bb - 1;
            l = l + (int64_t)a;
            const uint64_t d = (uint64_t)(h - l);
            const int sh = bitlen64(d);
            kk = prec - sh;
            e = kk > 0 ? (uint64_t)l >> sh : 0;
            l = (int64_t)(((uint64_t)l - (e << sh)) << kk);
            h = l + (int64_t)((d + 1) << kk) - 1;
            const int off0 = (int)(st.L & 63);
            const int avail = off0 ? 64 - off0 : 0;
            if (__builtin_expect(kk > avail, 0)) break;
            st.wc |= (e >> kk) << ((64 - off0) & 63);
            st.wa |= (e & ((1ull << kk) - 1)) << ((64 - off0 - kk) & 63);
            st.L += (uint64_t)kk;
        }
        if (i >= n) break;
        if constexpr (FT) {
            if (fudged) break;                              // step i for the general loop
        }
        if (!plane_append(st.L, st.wa, st.wc, kk, e, sp.cap_words, store)) {   // step i's crossing
            st.err = LAC_E_CAPACITY;
            ok = false;
            break;
        }
        i++;
    }
    st.nsym = nsym0 + i;
    return i;
}

// k_encode: one wave per stream over a chunk of steps; lane i prefetches the
// RowStats of step g0 + i, 64 steps at a time.  MAP: the mapping (LAC_MAP_*) as a
// compile-time constant (the launch passes it as `mapping` too), so the uniform chain's
// ceil / floor choice folds away instead of becoming a lane-mask select.
template <typename E, int MAP>
__global__ __launch_bounds__(256) void k_encode(const RowStats *__restrict__ stats, const int32_t *__restrict__ sym,
                                                int64_t B, int64_t t0, int64_t nsteps, const E *pmf,
                                                int64_t step_stride, int64_t stream_stride, int64_t V, int prec,
                                                EncState *states, uint64_t *planeA, uint64_t *planeC,
                                                uint64_t cap_words, uint64_t *trace, int mapping,
                                                bool allow_fudge) {
    const int lane = (int)lane_id();
    // (the stream index provably wave-uniform: the row and trace addresses -- and the
    // per-step trace test -- stay on the scalar unit)
    const int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + wave_in_block();
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
    // probe builds (-DLAC_ENC_PHASES=1, tools/enc_phase_probe.py): 0 the step's stats out of
    // the prefetch lanes, 1..3 coder_step's phases, 4 the per-64-step prefetch block
#if LAC_ENC_PHASES
    PhaseClock clock, *clk = &clock;
    clock.start();
#else
    NoClock *clk = nullptr;
#endif
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
        // (totals of 2^62 and more divide instead: frac_mul_div's uniform form needs T < 2^62)
        const bool frac_ok = lane < n && !(my.tot >> 62);
        const uint64_t flo = frac_ok ? row_frac(my.lo, my.tot) : kNoFrac;
        const uint64_t fhi = frac_ok ? row_frac(my.hi, my.tot) : kNoFrac;
        int i0 = 0;                                       // the first step the general loop takes
#if LAC_ENC_STRAIGHT
        if constexpr (sizeof(E) == 8) {
            // u64 tables: the straight form of straight_steps -- every step's row with
            // 0 < T < 2^62, a positive width at the symbol (for the floor mapping also
            // T <= 2^(prec-1) (hi - lo), so its two quotients differ by >= 1) and an in-range
            // symbol, and the state's width in (2^(prec-1), 2^prec]: no step can then meet a
            // zero width unfudged or leave that width range, and only rows with
            // T > 2^(prec-1) can fudge -- a fudged step leaves for the general loop below,
            // which takes the rest of the block.  (The u32 kernel keeps only the form below:
            // written beside these, its loop compiled ~3 % slower, profiles/r05/straight/.)
            const uint64_t half = 1ull << (prec - 1);
            const bool lfast = lane >= n || (frac_ok && my.tot != 0 && my.hi > my.lo && (uint32_t)mys < (uint32_t)V &&
                                             (MAP != LAC_MAP_FLOOR || ((my.tot - 1) >> (prec - 1)) < my.hi - my.lo));
            const uint64_t d0 = (uint64_t)(h - l);
            if (!trace && prec <= 61 && __ballot(!lfast) == 0 && nonneg_uni((int64_t)(d0 - half)) &&
                !(d0 >> prec)) {
                constexpr bool CEIL = MAP != LAC_MAP_FLOOR;
                const bool t32 = __ballot(lane < n && (my.tot >> 32)) == 0;
                const bool ft = CEIL && __ballot(lane < n && my.tot > half) != 0;   // a row that can fudge
                uint64_t ftl = 0;
                if (ft) {
                    ftl = lane < n && my.minp ? div_floor((u128)my.tot + (my.minp - 1), my.minp) : 0;
                    ftl = ftl < (1ull << 62) ? ftl : (1ull << 62);
                }
                SP sp{my.lo, my.hi, my.tot, flo, fhi, ftl, n, prec, cap_words, pa, pc, lane};
                if (t32)
                    i0 = ft ? straight_steps<CEIL, true, true>(sp, st, l, h, ok)
                            : straight_steps<CEIL, true, false>(sp, st, l, h, ok);
                else
                    i0 = ft ? straight_steps<CEIL, false, true>(sp, st, l, h, ok)
                            : straight_steps<CEIL, false, false>(sp, st, l, h, ok);
                if (!ok || i0 >= n) continue;
            }
        }
        // The block's straight form: when every step's row has 0 < T <= 2^(prec-1) < 2^32, a
        // positive width at the symbol and an in-range symbol, and the state's width is in
        // (2^(prec-1), 2^prec] (every renormalised state's is), no step can fudge
        // (T <= w minp), hit a zero width (w > T, so the two mul-divs differ by >= 1) or
        // leave that width range, so the 64 steps need none of coder_step's tests: per
        // step two mul-divs in 32 x 64-bit products, a branch-free renormalisation and the
        // plane append's one-word case, one rarely taken branch (the append crossing a
        // word).  Results, registers and error steps are coder_step's.
        if (i0 == 0) {
            const uint64_t half = 1ull << (prec - 1);
            const bool lfast = lane >= n || (frac_ok && my.tot != 0 && my.tot <= half && !(my.tot >> 32) &&
                                             my.hi > my.lo && (uint32_t)mys < (uint32_t)V);
            const uint64_t d0 = (uint64_t)(h - l);
            if (!trace && prec <= 61 && __ballot(!lfast) == 0 && nonneg_uni((int64_t)(d0 - half)) &&
                !(d0 >> prec)) {
                constexpr bool CEIL = MAP != LAC_MAP_FLOOR;
                const int64_t nsym0 = st.nsym;
                auto store = [&](uint64_t idx, uint64_t wa, uint64_t wc) {
                    if (lane == 0) { pa[idx] = wa; pc[idx] = wc; }
                };
                // step i's row values out of lane i (LAC_ENC_PIPE: read one step ahead, so
                // the readlanes' latency is not on the chain)
                auto rd = [&](int j, uint32_t &lo, uint32_t &hi, uint32_t &T, uint64_t &fl, uint64_t &fh) {
                    lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)my.lo, j);
                    hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)my.hi, j);
                    T = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)my.tot, j);
                    fl = readlane_u64(flo, j);
                    fh = readlane_u64(fhi, j);
                };
                uint32_t nlo, nhi, nT;
                uint64_t nfl, nfh;
                if constexpr (LAC_ENC_PIPE) rd(0, nlo, nhi, nT, nfl, nfh);
                int i = 0;
                int kk = 0;
                uint64_t e = 0;
                // the inner loop leaves only at the block's end or at a step whose digits
                // cross a plane word (~1 step in 7), whose append runs below it; one exit
                // test per step, no other branch
                while (i < n) {
                    for (; i < n; i++) {
                        uint32_t lo, hi, T;
                        uint64_t fl, fh;
                        if constexpr (LAC_ENC_PIPE) {
                            lo = nlo, hi = nhi, T = nT, fl = nfl, fh = nfh;
                            rd(i + 1 < n ? i + 1 : i, nlo, nhi, nT, nfl, nfh);
                        } else {
                            rd(i, lo, hi, T, fl, fh);
                        }
                        const uint64_t w = (uint64_t)(h - l + 1);
                        const uint64_t a = frac_mul_div32<CEIL>(fl, lo, w, T), bb = frac_mul_div32<CEIL>(fh, hi, w, T);
                        h = l + (int64_t)bb - 1;
                        l = l + (int64_t)a;
                        // renorm() without its kk <= 0 branch: kk = 0 keeps l and h (e = 0)
                        const uint64_t d = (uint64_t)(h - l);
                        const int sh = bitlen64(d);
                        kk = prec - sh;
                        e = kk > 0 ? (uint64_t)l >> sh : 0;
                        l = (int64_t)(((uint64_t)l - (e << sh)) << kk);
                        h = l + (int64_t)((d + 1) << kk) - 1;
                        // plane_append's case of digits inside the word of bit L-1 (or none)
                        const int off0 = (int)(st.L & 63);
                        const int avail = off0 ? 64 - off0 : 0;
                        if (__builtin_expect(kk > avail, 0)) break;
                        st.wc |= (e >> kk) << ((64 - off0) & 63);
                        st.wa |= (e & ((1ull << kk) - 1)) << ((64 - off0 - kk) & 63);
                        st.L += (uint64_t)kk;
                    }
                    if (i >= n) break;
                    if (!plane_append(st.L, st.wa, st.wc, kk, e, cap_words, store)) {   // step i's crossing
                        st.err = LAC_E_CAPACITY;
                        ok = false;
                        break;
                    }
                    i++;
                }
                st.nsym = nsym0 + i;
                continue;
            }
        }
#endif
        uint64_t fthr = lane < n && my.minp ? div_floor((u128)my.tot + (my.minp - 1), my.minp) : 0;
        fthr = fthr < (1ull << 62) ? fthr : (1ull << 62);   // w <= 2^61: w < fthr unchanged (coder_step's sign test)
        if (clk) clk->mark(4);
        for (int i = i0; i < n; i++) {
            const uint64_t lo = readlane_u64(my.lo, i), hi = readlane_u64(my.hi, i);
            const uint64_t T = readlane_u64(my.tot, i), minp = readlane_u64(my.minp, i);
            const uint64_t invb = readlane_u64(__builtin_bit_cast(uint64_t, my.inv_tot), i);
            const uint64_t fl = readlane_u64(flo, i), fh = readlane_u64(fhi, i), ft = readlane_u64(fthr, i);
            const int64_t s = __builtin_amdgcn_readlane(mys, i);
            const int64_t t = t0 + g0 + i;
            const E *row = pmf + t * step_stride + b * stream_stride;
            if (clk) clk->mark(0);
            if (!coder_step<E, true>(st, l, h, lo, hi, T, minp, s, row, V, prec, pa, pc, cap_words,
                                     trace ? trace + 2 * (t * B + b) : nullptr, lane, MAP,
                                     __builtin_bit_cast(double, invb), allow_fudge, fl, fh, ft, clk)) {
                ok = false;
                break;
            }
        }
    }
    if (lane == 0) store_state(st, l, h, pa, pc, cap_words, &states[b]);
#if LAC_ENC_PHASES
    if (lane == 0) {
        for (int k = 0; k < 5; k++) atomicAdd(&g_enc_phase[k], (unsigned long long)clock.acc[k]);
        atomicAdd(&g_enc_phase[6], (unsigned long long)st.nsym);
    }
#endif
}

// ------------------------------------------------------------------ fused path
// k_encode_fused: one wave owns one stream for the whole call.  Per step it scans
// the row (HBM-bound) and applies the range update in registers, so no per-row
// statistics round-trip through HBM and no second launch; with kReset/kFinish
// the stream is also initialised and flushed + packed in the same launch.  With
// >= 2048 streams there are >= 8 waves per CU streaming rows, which hides each
// wave's short serial coder step behind the others' loads.

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

}  // namespace


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
            if (c->mapping == LAC_MAP_FLOOR)
                k_encode<E, LAC_MAP_FLOOR><<<blocks, 64 * kWavesPerBlock, 0, st>>>(
                    c->stats, sym, c->B, t0, n, pmf, step_stride, stream_stride, c->V, c->prec, c->enc, c->planeA,
                    c->planeC, c->cap_words, trace, c->mapping, true);
            else
                k_encode<E, LAC_MAP_CEIL><<<blocks, 64 * kWavesPerBlock, 0, st>>>(
                    c->stats, sym, c->B, t0, n, pmf, step_stride, stream_stride, c->V, c->prec, c->enc, c->planeA,
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


// ---- launchers for the logits path's encode (lac_logits.hip q1_encode): k_encode over
// the q1 row statistics, fudge disabled (q1 rows cannot fudge)
int enc_reset_launch(lac_ctx *c, hipStream_t st) {
    k_enc_reset<<<(unsigned)((c->B + 255) / 256), 256, 0, st>>>(c->enc, c->B, c->prec);
    CHECK_LAUNCH();
    return LAC_OK;
}

int enc_stats_launch(lac_ctx *c, const int32_t *sym, int64_t t0, int64_t n, uint64_t *trace, hipStream_t st) {
    const unsigned blocks = (unsigned)((c->B + kWavesPerBlock - 1) / kWavesPerBlock);
    {
        ProfScope ps(c, KID_ENCODE, st);
        k_encode<uint32_t, LAC_MAP_CEIL><<<blocks, 64 * kWavesPerBlock, 0, st>>>(
            c->stats, sym, c->B, t0, n, (const uint32_t *)nullptr, 0, 0, c->V, c->prec, c->enc, c->planeA,
            c->planeC, c->cap_words, trace, LAC_MAP_CEIL, false);
    }
    CHECK_LAUNCH();
    return LAC_OK;
}

int enc_finish_launch(lac_ctx *c, int term, hipStream_t st) {
    ProfScope ps(c, KID_FINISH, st);
    k_finish<<<(unsigned)((c->B + 255) / 256), 256, 0, st>>>(c->enc, c->planeA, c->planeC, c->cap_words, c->B,
                                                             c->prec, c->nbits, term);
    CHECK_LAUNCH();
    return LAC_OK;
}

extern "C" {

#if LAC_ENC_PHASES
// probe builds only (tools/enc_phase_probe.py): k_encode's phase cycle sums (s_memtime)
// and the symbols they cover; reset != 0 clears them
int lac_debug_enc_phases(uint64_t *out8, int reset) {
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_enc_phase), sizeof(uint64_t) * 8));
    if (reset) {
        const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_enc_phase), z, sizeof z));
    }
    return LAC_OK;
}
#endif

int lac_encode_reset(lac_ctx *c, void *stream) {
    if (!c) return fail(LAC_E_ARG, "ctx is NULL");
    HIPCHK(hipSetDevice(c->device));
    c->mode = 0;
    c->finished = 0;
    c->open = 0;
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
    if (rc == LAC_OK && steps > 0) enc_mark_open(c);
    return rc;
}

int lac_encode_job(lac_ctx *c, const void *pmf_dev, int64_t step_stride, int64_t stream_stride,
                   const int32_t *sym_dev, int64_t steps, uint64_t *trace_dev, void *stream) {
    const int rc = encode_dispatch(c, pmf_dev, step_stride, stream_stride, sym_dev, steps, trace_dev, stream,
                                   kReset | kFinish);
    if (rc == LAC_OK) enc_mark_finished(c);
    return rc;
}

int lac_encode_finish(lac_ctx *c, void *stream) {
    if (!c) return fail(LAC_E_ARG, "ctx is NULL");
    if (c->mode != 0) return fail(LAC_E_STATE, "context is decoding");
    HIPCHK(hipSetDevice(c->device));
    ProfScope ps(c, KID_FINISH, S(stream));
    enc_mark_finished(c);
    k_finish<<<(unsigned)((c->B + 255) / 256), 256, 0, S(stream)>>>(c->enc, c->planeA, c->planeC, c->cap_words, c->B,
                                                                   c->prec, c->nbits, c->term);
    CHECK_LAUNCH();
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
    // Only between jobs: an open encode has written part of its planes to the current
    // buffers, and k_finish would carry-add over the new ones (silently wrong bytes).
    if (c->mode != 0) return fail(LAC_E_STATE, "context is decoding; redirect the output between encode jobs");
    if (c->open)
        return fail(LAC_E_STATE, "streams hold coded symbols that are not finished: redirect the output before "
                                 "the job's first encode call or after lac_encode_finish / lac_encode_reset");
    c->planeA = planeA_dev ? planeA_dev : c->own_planeA;
    c->nbits = nbits_dev ? nbits_dev : c->own_nbits;
    // finished again exactly when the new buffers are the ones the last finished job went to
    c->finished = c->fin_planeA && c->planeA == c->fin_planeA && c->nbits == c->fin_nbits;
    return LAC_OK;
}

int lac_pack_bits(lac_ctx *c, uint8_t *dst, int hdr_bytes, uint64_t *len_dev, void *stream) {
    if (!len_dev) return fail(LAC_E_ARG, "bad argument");
    return lac_pack_bits_at(c, dst, ~0ull, hdr_bytes, nullptr, len_dev, nullptr, stream);
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
    bool coded = false;
    for (int64_t b = 0; b < c->B; b++) coded = coded || host_in[b].nsym > 0 || host_in[b].L > 0;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpyAsync(c->enc, host_in, sizeof(EncState) * c->B, hipMemcpyHostToDevice, S(stream)));
    if (planes_host) {
        const size_t n = sizeof(uint64_t) * c->cap_words * c->B;
        HIPCHK(hipMemcpyAsync(c->planeA, planes_host, n, hipMemcpyHostToDevice, S(stream)));
        HIPCHK(hipMemcpyAsync(c->planeC, planes_host + c->cap_words * c->B, n, hipMemcpyHostToDevice, S(stream)));
    }
    c->finished = 0;
    c->open = coded ? 1 : 0;
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

}  // extern "C"
