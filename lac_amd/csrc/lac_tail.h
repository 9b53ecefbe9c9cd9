// lac_tail.h -- the decoder's tail in the reference's own register frame
// (included by lac_decode.hip inside its kernel namespace; TailState is in lac_core.h).
//
// A_from_bin (/root/reference/arith_code.py:248-334) keeps l, h and the received
// window [lb, hb] (the bits so far padded with 0s / 1s).  The value-form decoders
// reproduce its symbols while the window lies inside [l, h]; two things need the
// window itself:
//
//   DECIDE  decide_symbol + emit_symbol + emit_bit (:268-291) on the final
//           window: ls = val_to_symbol(lb - l, w), hs = val_to_symbol(hb - l, w);
//           equal -> emit, renormalise l, h, lb, hb together; else undetermined.
//           Reproduces the reference where the window leaves [l, h] (corrupt or
//           foreign bits): AssertionError('unknown symbol', V) for table
//           predictors, out-of-range symbols for the uniform Predictor(n).
//   FLUSH   flush (:300-317): while not (lb <= l and h <= hb), emit the symbol of
//           largest overlap ratio k(s) = |[lb-l, hb-l] & range(s)| / |range(s)|
//           among ls..hs (a Python float; max() keeps the first maximum), with no
//           renormalisation, then reset the registers.  Raises where the
//           reference raises: a zero-width candidate (ZeroDivisionError in k), the
//           candidate V (AssertionError 'unknown symbol'), an empty overlap
//           (emit_symbol's AssertionError).
//
// One 256-thread block per stream and call; the row is streamed up to three
// times (totals; the counts of the (fudged) CDF at or below the two window
// targets; the candidates' ranges and the first zero-width candidate).  This is
// a once-per-stream tail: it is written for exactness, not bandwidth.
//
// Candidate ranking without floats over the row: interior candidates
// ls < s < hs lie inside the window (val_to_symbol and symbol_to_range are
// inverse on [0, w) for the ceil mapping; for the floor mapping of Predictor(n)
// the window still covers them), so their ratio is exactly 1.0 -- only
// k(ls) and k(hs) need computing (lac_core.h cr_ratio, CPython's rounding).

enum { kTailDecide = 0, kTailFlush = 1 };
enum { kTailEmitted = 0, kTailIdle = 1 };   // code_out >= 0: a symbol / nothing (undetermined or flushed)
constexpr int64_t kTailStillLimit = 1000;   // emits leaving [l, h] unchanged: the reference loops forever

constexpr int kTailThreads = 256;

__device__ inline i128 i128_min(i128 a, i128 b) { return a < b ? a : b; }
__device__ inline i128 i128_max(i128 a, i128 b) { return a > b ? a : b; }
__device__ inline i128 overlap128(i128 a, i128 b, i128 c, i128 d) {        // region_overlap, :59-61
    const i128 r = i128_min(d, b) - i128_max(a, c) + 1;
    return r > 0 ? r : 0;
}

// Block-wide helpers (kTailThreads threads, LDS scratch from the caller).
__device__ inline u128 tail_block_sum_u128(u128 v, u128 *sh) {
    v = wave_sum_u128(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[w] = v;
    __syncthreads();
    u128 t = 0;
    for (int i = 0; i < kTailThreads / 64; i++) t += sh[i];
    return t;
}
__device__ inline uint64_t tail_block_min_u64(uint64_t v, uint64_t *sh) {
    v = wave_min_u64(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[w] = v;
    __syncthreads();
    uint64_t t = ~0ull;
    for (int i = 0; i < kTailThreads / 64; i++) t = sh[i] < t ? sh[i] : t;
    return t;
}
// inclusive scans; *total receives the block's total / maximum
__device__ inline uint64_t tail_block_scan_u64(uint64_t v, uint64_t *sh, uint64_t *total) {
    const uint64_t in = wave_incl_scan_u64(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 63) sh[w] = in;
    __syncthreads();
    uint64_t before = 0, t = 0;
    for (int i = 0; i < kTailThreads / 64; i++) {
        if (i < w) before += sh[i];
        t += sh[i];
    }
    *total = t;
    return before + in;
}
__device__ inline i128 tail_block_maxscan_i128(i128 v, i128 *sh, i128 *total) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const i128 o = shfl_i128(v, lane >= d ? lane - d : lane);
        v = (lane >= d && o > v) ? o : v;
    }
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 63) sh[w] = v;
    __syncthreads();
    i128 before = kI128Min, t = kI128Min;
    for (int i = 0; i < kTailThreads / 64; i++) {
        if (i < w) before = i128_max(before, sh[i]);
        t = i128_max(t, sh[i]);
    }
    *total = t;
    return i128_max(before, v);
}

// The (possibly fudged) CDF entry dist'_i from the running sum c_i and the running
// maximum of X_j = c_j*w - j*T (fudged_dist in closed form, lac_core.h fudge_f;
// here for any w, including w < V, where the clamp w - V + 1 drops below 1).
__device__ inline uint64_t tail_dist(bool fudged, int64_t i, uint64_t c, i128 xmax, uint64_t T, uint64_t w,
                                     int64_t V) {
    if (!fudged) return c;
    const int64_t cap = (int64_t)w - V + 1;
    uint64_t g = 1;
    if (cap > 1 && xmax >= (i128)2 * (i128)T) {
        const uint64_t m = div_floor((u128)xmax, T);      // <= w
        g = (int64_t)m < cap ? m : (uint64_t)cap;
    }
    return (uint64_t)i + g;
}

struct TailPick {
    int code;          // 0 symbol chosen, kTailIdle undetermined, < 0 error (LAC_E_*)
    i128 s, r0, r1;    // symbol and its range [r0, r1) relative to l
    int64_t err_sym;   // the symbol an 'unknown symbol' error names
};

// Ceil mapping on a table row (CDFPredictor.val_to_symbol / symbol_to_range with
// fudged_dist, :83-110), all 256 threads.
template <typename E>
__device__ TailPick tail_pick_table(const E *row, int64_t V, int mode, int64_t va, int64_t vb, uint64_t w) {
    __shared__ u128 sh128[kTailThreads / 64];
    __shared__ uint64_t sh64[kTailThreads / 64];
    __shared__ i128 shx[kTailThreads / 64];
    __shared__ uint64_t dchunk[kTailThreads];
    __shared__ uint64_t cap[5];                          // dist' at ls-1, ls, ls+1, hs-1, hs
    __shared__ int64_t zfirst;
    const int tid = threadIdx.x;
    TailPick p{0, 0, 0, 0, 0};
    // pass 1: T and the positive minimum (CDFPredictor.minp, :79-82)
    u128 tsum = 0;
    uint64_t kmin = ~0ull;
    for (int64_t i = tid; i < V; i += kTailThreads) {
        const uint64_t x = (uint64_t)row[i];
        tsum += x;
        const uint64_t k = x - 1;                        // 0 wraps to the maximum
        kmin = k < kmin ? k : kmin;
    }
    const u128 T128 = tail_block_sum_u128(tsum, sh128);
    const uint64_t minp = tail_block_min_u64(kmin, sh64) + 1;
    if (T128 == 0 || (T128 >> 64)) { p.code = LAC_E_TABLE; return p; }
    const uint64_t T = (uint64_t)T128;
    const bool fudged = is_fudged(T, w, minp);
    const uint64_t d = fudged ? ((uint64_t)V > w ? (uint64_t)V : w) : T;   // dist'[-1]
    // targets (v * d) // w of the window ends; v < 0 -> below every entry, v >= w -> above
    auto target = [&](int64_t v, bool *below, bool *above) -> uint64_t {
        *below = v < 0;
        *above = v >= (int64_t)w;
        return (*below || *above) ? 0 : div_floor((u128)(uint64_t)v * d, w);
    };
    bool ba, aa, bb, ab;
    const uint64_t ta = target(va, &ba, &aa), tb = target(vb, &bb, &ab);
    // pass 2: ls, hs = bisect_right(dist', t) = #{i : dist'_i <= t}
    uint64_t na = 0, nb = 0, carry = 0;
    i128 xcarry = kI128Min;
    for (int64_t base = 0; base < V; base += kTailThreads) {
        const int64_t i = base + tid;
        const uint64_t x = i < V ? (uint64_t)row[i] : 0;
        uint64_t tot;
        const uint64_t c = carry + tail_block_scan_u64(x, sh64, &tot);
        carry += tot;
        i128 xm = kI128Min;
        if (fudged) {
            i128 xt;
            xm = i128_max(xcarry, tail_block_maxscan_i128(i < V ? fudge_x(c, i, w, T) : kI128Min, shx, &xt));
            xcarry = i128_max(xcarry, xt);
        }
        if (i < V) {
            const uint64_t dv = tail_dist(fudged, i, c, xm, T, w, V);
            na += (!ba && !aa && dv <= ta) ? 1 : 0;
            nb += (!bb && !ab && dv <= tb) ? 1 : 0;
        }
    }
    const int64_t ls = ba ? 0 : aa ? V : (int64_t)(uint64_t)tail_block_sum_u128(na, sh128);
    const int64_t hs = bb ? 0 : ab ? V : (int64_t)(uint64_t)tail_block_sum_u128(nb, sh128);
    if (mode == kTailDecide && ls != hs) { p.code = kTailIdle; return p; }
    // pass 3: dist' around ls and hs, and the first zero-width candidate (flush's k)
    if (tid < 5) cap[tid] = 0;
    if (tid == 0) zfirst = V;
    const int64_t hv = hs < V ? hs : V - 1;
    const int64_t want[5] = {ls - 1, ls, ls + 1, hs - 1, hs};
    carry = 0;
    xcarry = kI128Min;
    uint64_t prev_last = 0;                              // dist' of the entry before this chunk
    for (int64_t base = 0; base <= hv && base < V; base += kTailThreads) {
        const int64_t i = base + tid;
        const uint64_t x = i < V ? (uint64_t)row[i] : 0;
        uint64_t tot;
        const uint64_t c = carry + tail_block_scan_u64(x, sh64, &tot);
        carry += tot;
        i128 xm = kI128Min;
        if (fudged) {
            i128 xt;
            xm = i128_max(xcarry, tail_block_maxscan_i128(i < V ? fudge_x(c, i, w, T) : kI128Min, shx, &xt));
            xcarry = i128_max(xcarry, xt);
        }
        const uint64_t dv = i < V ? tail_dist(fudged, i, c, xm, T, w, V) : 0;
        dchunk[tid] = dv;
        __syncthreads();
        const uint64_t dprev = tid ? dchunk[tid - 1] : prev_last;
        if (i < V) {
#pragma unroll
            for (int k = 0; k < 5; k++)
                if (i == want[k]) cap[k] = dv;
            if (mode == kTailFlush && i >= ls && i <= hv) {
                const uint64_t lo = i ? div_ceil((u128)dprev * w, d) : 0, hi = div_ceil((u128)dv * w, d);
                if (hi == lo) atomicMin((unsigned long long *)&zfirst, (unsigned long long)i);
            }
        }
        const uint64_t last = dchunk[kTailThreads - 1];
        __syncthreads();
        prev_last = last;
    }
    __syncthreads();
    if (tid != 0) return p;
    auto range = [&](int64_t s, uint64_t dsm1, uint64_t ds, i128 *r0, i128 *r1) {   // symbol_to_range, :98-110
        *r0 = s ? (i128)div_ceil((u128)dsm1 * w, d) : 0;
        *r1 = (i128)div_ceil((u128)ds * w, d);
    };
    if (mode == kTailDecide) {                           // ls == hs: emit_symbol(ls)
        if (ls >= V) { p.code = LAC_E_SYMBOL_RANGE; p.err_sym = ls; return p; }
        p.s = ls;
        range(ls, cap[0], cap[1], &p.r0, &p.r1);
        return p;
    }
    if (zfirst < V) { p.code = LAC_E_FLUSH_ZERO_WIDTH; return p; }          // k(s): division by zero
    if (hs >= V) { p.code = LAC_E_SYMBOL_RANGE; p.err_sym = V; return p; }   // k(V): unknown symbol
    i128 a0, a1;
    range(ls, cap[0], cap[1], &a0, &a1);
    p.s = ls; p.r0 = a0; p.r1 = a1;
    if (ls == hs) return p;
    const double kl = cr_ratio((uint64_t)overlap128(va, vb, a0, a1 - 1), (uint64_t)(a1 - a0));
    if (kl == 1.0) return p;
    if (hs - ls >= 2) {                                  // an interior candidate: ratio exactly 1.0
        range(ls + 1, cap[1], cap[2], &p.r0, &p.r1);
        p.s = ls + 1;
        return p;
    }
    i128 b0, b1;
    range(hs, cap[3], cap[4], &b0, &b1);
    const double kh = cr_ratio((uint64_t)overlap128(va, vb, b0, b1 - 1), (uint64_t)(b1 - b0));
    if (kh > kl) { p.s = hs; p.r0 = b0; p.r1 = b1; }
    return p;
}

// Floor mapping of the uniform Predictor(n) (:64-74): val_to_symbol = (v*n)//denom,
// symbol_to_range = (s*denom//n, (s+1)*denom//n) for ANY integer s (no range check).
__device__ inline TailPick tail_pick_uniform(int64_t n, int mode, int64_t va, int64_t vb, uint64_t w) {
    TailPick p{0, 0, 0, 0, 0};
    const i128 ls = floordiv_i128((i128)va * n, w);
    const i128 hs = floordiv_i128((i128)vb * n, w);
    auto lo = [&](i128 s) { return floordiv_i128(s * (i128)w, (uint64_t)n); };
    if (mode == kTailDecide && ls != hs) { p.code = kTailIdle; return p; }
    p.s = ls; p.r0 = lo(ls); p.r1 = lo(ls + 1);
    if (mode == kTailDecide || ls == hs) {
        if (mode == kTailFlush && p.r1 == p.r0) p.code = LAC_E_FLUSH_ZERO_WIDTH;
        return p;
    }
    // widths are 0 or 1 once w < n: some candidate has none iff they sum to fewer than the count
    if (w < (uint64_t)n && lo(hs + 1) - lo(ls) < hs - ls + 1) { p.code = LAC_E_FLUSH_ZERO_WIDTH; return p; }
    const double kl = cr_ratio((uint64_t)overlap128(va, vb, p.r0, p.r1 - 1), (uint64_t)(p.r1 - p.r0));
    if (kl == 1.0) return p;
    if (hs - ls >= 2) { p.s = ls + 1; p.r0 = lo(ls + 1); p.r1 = lo(ls + 2); return p; }
    const i128 b0 = lo(hs), b1 = lo(hs + 1);
    const double kh = cr_ratio((uint64_t)overlap128(va, vb, b0, b1 - 1), (uint64_t)(b1 - b0));
    if (kh > kl) { p.s = hs; p.r0 = b0; p.r1 = b1; }
    return p;
}

// One DECIDE or FLUSH step of every stream.  sym_out[b] / code_out[b]: the symbol
// and kTailEmitted, kTailIdle (undetermined / flushed, nothing emitted), or the
// stream's sticky error (< 0).
template <typename E>
__global__ __launch_bounds__(kTailThreads) void k_decode_tail(const E *__restrict__ pmf, int64_t stream_stride,
                                                              int64_t V, int prec, int mapping, int mode,
                                                              TailState *states, int64_t *sym_out,
                                                              int32_t *code_out) {
    const int64_t b = blockIdx.x;
    const TailState st0 = states[b];                     // block-uniform
    const int64_t D = (int64_t)1 << prec, H = (int64_t)1 << (prec - 1);
    auto finish = [&](const TailState &st, int code, int64_t s) {
        if (threadIdx.x == 0) {
            states[b] = st;
            sym_out[b] = s;
            code_out[b] = code;
        }
    };
    if (st0.err) { finish(st0, st0.err, 0); return; }
    if (st0.done) { finish(st0, kTailIdle, 0); return; }
    if (mode == kTailFlush && st0.lb <= st0.l && st0.h <= st0.hb) {      // :308, then the reset :314-317
        TailState st = st0;
        st.l = 0; st.h = D - 1; st.lb = 0; st.hb = D - 1; st.done = 1;
        finish(st, kTailIdle, 0);
        return;
    }
    const uint64_t w = (uint64_t)(st0.h - st0.l + 1);
    const int64_t va = st0.lb - st0.l, vb = st0.hb - st0.l;
    TailPick p;
    if (mapping == LAC_MAP_FLOOR) {
        if (threadIdx.x != 0) return;
        p = tail_pick_uniform(V, mode, va, vb, w);
    } else {
        p = tail_pick_table<E>(pmf + b * stream_stride, V, mode, va, vb, w);
        if (threadIdx.x != 0) return;
    }
    TailState st = st0;
    if (p.code == kTailIdle) { finish(st, kTailIdle, 0); return; }
    if (p.code < 0) {
        st.err = p.code;
        finish(st, p.code, p.err_sym);
        return;
    }
    // emit_symbol (:274-283): the range must meet the window
    const i128 nl = (i128)st.l + p.r0, nh = (i128)st.l + p.r1 - 1;
    const i128 lim = (i128)1 << 62;
    if (overlap128(nl, nh, st.lb, st.hb) == 0 || p.s >= lim || p.s <= -lim || nl <= -lim || nh >= lim) {
        st.err = (overlap128(nl, nh, st.lb, st.hb) == 0) ? LAC_E_DECODE_RANGE : LAC_E_ARG;
        finish(st, st.err, 0);
        return;
    }
    const bool same = nl == st.l && nh == st.h;
    st.l = (int64_t)nl;
    st.h = (int64_t)nh;
    st.nsym++;
    if (mode == kTailDecide) {
        while (st.h - st.l < H) {                        // emit_bit (:284-291)
            const int64_t dd = floordiv_pos(st.l, H);
            st.l = st.l * 2 - dd * D;
            st.h = st.h * 2 + 1 - dd * D;
            st.lb = st.lb * 2 - dd * D;
            st.hb = st.hb * 2 + 1 - dd * D;
        }
    } else {
        st.still = same ? st.still + 1 : 0;
        if (st.still >= kTailStillLimit) {
            st.err = LAC_E_FLUSH_LOOP;
            finish(st, st.err, (int64_t)p.s);
            return;
        }
    }
    finish(st, kTailEmitted, (int64_t)p.s);
}

// Value-form registers -> the reference frame: lb = x (the window read with 0s
// past the end), hb = x + 2^u - 1 with u the window bits past the end.
__global__ void k_decode_tail_begin(const DecState *dec, const uint64_t *nbits, int64_t B, int prec,
                                    TailState *out) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const DecState d = dec[b];
    TailState t;
    t.l = d.l;
    t.h = d.h;
    const uint64_t past = d.pos > nbits[b] ? d.pos - nbits[b] : 0;
    const int u = past < (uint64_t)prec ? (int)past : prec;
    t.lb = d.x;
    t.hb = d.x + (((int64_t)1 << u) - 1);
    t.err = d.err ? d.err : (d.det ? 0 : LAC_E_STATE);
    t.done = 0;
    t.still = 0;
    t.nsym = 0;
    out[b] = t;
}
