/*
 * lac_oracle.c -- CPU restatement of the reference arithmetic coder.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the checker for the HIP product path
 * (lac_amd/csrc): only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it (via oracle/oracle.py).  Nothing in the product
 * links or calls it.
 *
 * It is a deliberately *literal* restatement of
 *   /root/reference/arith_code.py   A_to_bin (:156-246), A_from_bin value form,
 *                                   CDFPredictor (:76-110), region_overlap (:59-61)
 *   /root/reference/arithmetic_coding.py  ACSampler encode (:50-56, :73-95),
 *                                   Region (:128-177), CarryBuffer (:180-208)
 * on exact integers (unsigned __int128 where the reference relies on Python
 * big ints).  Per step it rebuilds the CDF and positive minimum in O(V) exactly
 * as CDFPredictor does, runs the fudge loop literally (:83-93) and renormalises
 * one digit at a time (:176-192).  It is pinned against vectors produced by the
 * reference itself (tests/golden, tests/test_oracle_golden.py).
 *
 * Status codes mirror include/lac.h (the product header is not included so that
 * the oracle stays independent of the thing it checks).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* The q1 exp table is a format constant (the quantiser's definition), shared
 * with the product; the arithmetic below is an independent restatement. */
#include "../include/lac_q1_table.h"
static const uint32_t Q1_TAB[LAC_Q1_TAB_SIZE] = LAC_Q1_TAB_INIT;

typedef unsigned __int128 u128;
typedef __int128 i128;

enum {
    R_OK = 0, R_E_ARG = -1, R_E_PREC = -2, R_E_SYMBOL_RANGE = -3, R_E_ZERO_WIDTH = -4,
    R_E_TABLE = -5, R_E_DECODE_RANGE = -6, R_E_CAPACITY = -7
};

static inline uint64_t ld(const void *row, int eb, int64_t i) {
    return eb == 4 ? ((const uint32_t *)row)[i] : ((const uint64_t *)row)[i];
}

static inline int64_t floordiv(int64_t a, int64_t b) {       /* Python // for b > 0 */
    int64_t q = a / b;
    if ((a % b) != 0 && (a < 0)) q -= 1;
    return q;
}

/* region_overlap, arith_code.py:59-61 (closed intervals). */
static inline int64_t region_overlap(int64_t a, int64_t b, int64_t c, int64_t d) {
    int64_t hi = d < b ? d : b, lo = a > c ? a : c;
    int64_t r = hi - lo + 1;
    return r > 0 ? r : 0;
}

/* Build the inclusive CDF (ProbPredictor.calc_dist :117-123) and the positive
 * minimum (CDFPredictor.minp :79-82).  Fails if the total leaves u64 or is 0. */
static int build_cdf(const void *row, int eb, int64_t V, uint64_t *cdf, uint64_t *minp) {
    u128 c = 0;
    uint64_t m = 0;
    for (int64_t i = 0; i < V; i++) {
        uint64_t p = ld(row, eb, i);
        c += p;
        if (c >> 64) return R_E_TABLE;
        cdf[i] = (uint64_t)c;
        if (p > 0 && (m == 0 || p < m)) m = p;
    }
    if (c == 0) return R_E_TABLE;
    *minp = m;
    return R_OK;
}

/* fudged_dist, literal loop (arith_code.py:83-93).  dist == cdf when unfudged. */
static const uint64_t *fudged_dist(const uint64_t *cdf, uint64_t minp, int64_t V, uint64_t denom,
                                   uint64_t *scratch) {
    uint64_t T = cdf[V - 1];
    if ((u128)T <= (u128)denom * minp) return cdf;
    i128 p = 0;
    for (int64_t i = 0; i < V; i++) {
        i128 d = (i128)(((u128)cdf[i] * denom) / T) - p;
        i128 cap = (i128)denom - p - V + i + 1;
        if (cap < d) d = cap;
        if (d < 1) d = 1;
        p += d;
        scratch[i] = (uint64_t)p;
    }
    return scratch;
}

/* CDFPredictor.symbol_to_range (arith_code.py:98-110): ceil mapping. */
static int symbol_to_range(const uint64_t *dist, int64_t V, int64_t s, uint64_t denom,
                           uint64_t *lo, uint64_t *hi) {
    if (s >= V || s < 0) return R_E_SYMBOL_RANGE;
    uint64_t d = dist[V - 1];
    u128 ldn = (u128)(s > 0 ? dist[s - 1] : 0) * denom, hdn = (u128)dist[s] * denom;
    *lo = (uint64_t)((ldn + d - 1) / d);
    *hi = (uint64_t)((hdn + d - 1) / d);
    return R_OK;
}

/* CDFPredictor.val_to_symbol (arith_code.py:94-97): bisect_right(dist, v*d//denom). */
static int64_t val_to_symbol(const uint64_t *dist, int64_t V, uint64_t v, uint64_t denom) {
    uint64_t t = (uint64_t)(((u128)v * dist[V - 1]) / denom);
    int64_t lo = 0, hi = V;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (dist[mid] <= t) lo = mid + 1; else hi = mid;
    }
    return lo;
}

static int check_prec(int prec, int64_t V) {
    if (prec < 2 || prec > 61) return R_E_PREC;
    if ((int64_t)1 << (prec - 1) < V) return R_E_PREC;
    return R_OK;
}

/* Digits (signed, {-1..3}) -> MSB-first bytes of R = sum d_k 2^(L-1-k)
 * (A_to_bin.encode :212-219 == bits() :230-246), group_bits zero padding. */
static int digits_to_bytes(const int8_t *dg, uint64_t L, uint8_t *out, uint64_t cap_bytes) {
    uint64_t nbytes = (L + 7) / 8;
    if (nbytes > cap_bytes) return R_E_CAPACITY;
    memset(out, 0, nbytes);
    int64_t carry = 0;
    for (uint64_t k = L; k-- > 0;) {
        int64_t v = dg[k] + carry;
        int64_t bit = v & 1;                 /* floor mod 2 */
        carry = (v - bit) / 2;               /* exact: v - bit is even */
        if (bit) out[k >> 3] |= (uint8_t)(0x80u >> (k & 7));
    }
    return carry == 0 ? R_OK : R_E_ARG;      /* R < 2^L always holds for the reference */
}

typedef struct {
    const void *pmf; int eb; int64_t V, steps, step_stride; const int32_t *syms; int sym_stride;
    int prec; uint8_t *out; uint64_t cap_bytes; uint64_t *nbits; int8_t *digits; uint64_t cap_digits;
    uint64_t *ndigits; int64_t *fail_step;
} enc_job;

/* One stream: A_to_bin.run(symbols, stop=1) (arith_code.py:187-211). */
static int encode_one(const enc_job *j, uint64_t *cdf, uint64_t *scratch, int8_t *dg, uint64_t dcap) {
    int rc = check_prec(j->prec, j->V);
    if (rc) return rc;
    const int64_t P = j->prec, D = (int64_t)1 << P, Hd = (int64_t)1 << (P - 1);
    int64_t l = 0, h = D - 1;
    uint64_t L = 0;
    if (j->fail_step) *j->fail_step = -1;
    for (int64_t t = 0; t < j->steps; t++) {
        const void *row = (const char *)j->pmf + (size_t)(t * j->step_stride) * j->eb;
        uint64_t minp;
        if ((rc = build_cdf(row, j->eb, j->V, cdf, &minp))) goto fail;
        uint64_t w = (uint64_t)(h - l + 1);
        const uint64_t *dist = fudged_dist(cdf, minp, j->V, w, scratch);
        uint64_t a, b;
        if ((rc = symbol_to_range(dist, j->V, j->syms[t * j->sym_stride], w, &a, &b))) goto fail;
        if (a >= b) { rc = R_E_ZERO_WIDTH; goto fail; }        /* the reference hangs here */
        h = l + (int64_t)b - 1;
        l = l + (int64_t)a;
        while (h - l < Hd) {                                  /* decide_bit/emit_bit :176-186 */
            int64_t d = l / Hd;
            l = l * 2 - d * D;
            h = h * 2 + 1 - d * D;
            if (L >= dcap) { rc = R_E_CAPACITY; goto fail; }
            dg[L++] = (int8_t)d;
        }
        continue;
    fail:
        if (j->fail_step) *j->fail_step = t;
        return rc;
    }
    while (l > 0 || h + 1 < D) {                              /* flush :193-202 */
        int64_t d = floordiv(l, Hd);
        if (region_overlap(l, h, d * Hd, (d + 1) * Hd) < region_overlap(l, h, (d + 1) * Hd, (d + 2) * Hd))
            d += 1;
        l = l * 2 - d * D;
        h = h * 2 + 1 - d * D;
        if (L >= dcap) return R_E_CAPACITY;
        dg[L++] = (int8_t)d;
    }
    if (j->digits) {
        if (L > j->cap_digits) return R_E_CAPACITY;
        memcpy(j->digits, dg, L);
    }
    if (j->ndigits) *j->ndigits = L;
    *j->nbits = L;
    return digits_to_bytes(dg, L, j->out, j->cap_bytes);
}

static uint64_t digit_cap(const enc_job *j) { return (uint64_t)j->steps * (uint64_t)(j->prec + 2) + 64; }

int lacref_encode(const void *pmf, int elem_bytes, int64_t V, int64_t steps, int64_t step_stride,
                  const int32_t *syms, int prec, uint8_t *out, uint64_t cap_bytes, uint64_t *nbits,
                  int8_t *digits, uint64_t cap_digits, uint64_t *ndigits, int64_t *fail_step) {
    if (!pmf || !syms || !out || !nbits || V < 1 || steps < 0 || (elem_bytes != 4 && elem_bytes != 8))
        return R_E_ARG;
    enc_job j = {pmf, elem_bytes, V, steps, step_stride, syms, 1, prec, out, cap_bytes, nbits,
                 digits, cap_digits, ndigits, fail_step};
    uint64_t *cdf = malloc(sizeof(uint64_t) * V), *scr = malloc(sizeof(uint64_t) * V);
    uint64_t dcap = digit_cap(&j);
    int8_t *dg = malloc(dcap);
    int rc = (cdf && scr && dg) ? encode_one(&j, cdf, scr, dg, dcap) : R_E_ARG;
    free(cdf); free(scr); free(dg);
    return rc;
}

/* ---- batched encode over [steps][streams] rows, streams split over threads ---- */
typedef struct {
    const void *pmf; int eb; int64_t V, steps, streams, step_stride, stream_stride;
    const int32_t *syms; int prec; uint8_t *out; uint64_t cap_bytes; uint64_t *nbits; int32_t *status;
    int64_t b0, b1;
} batch_arg;

static void *batch_worker(void *vp) {
    batch_arg *a = vp;
    uint64_t *cdf = malloc(sizeof(uint64_t) * a->V), *scr = malloc(sizeof(uint64_t) * a->V);
    uint64_t dcap = (uint64_t)a->steps * (uint64_t)(a->prec + 2) + 64;
    int8_t *dg = malloc(dcap);
    for (int64_t b = a->b0; b < a->b1; b++) {
        enc_job j = {(const char *)a->pmf + (size_t)(b * a->stream_stride) * a->eb, a->eb, a->V, a->steps,
                     a->step_stride, a->syms + b, (int)a->streams, a->prec, a->out + (size_t)b * a->cap_bytes,
                     a->cap_bytes, a->nbits + b, NULL, 0, NULL, NULL};
        a->status[b] = (cdf && scr && dg) ? encode_one(&j, cdf, scr, dg, dcap) : R_E_ARG;
    }
    free(cdf); free(scr); free(dg);
    return NULL;
}

int lacref_encode_batch(const void *pmf, int elem_bytes, int64_t V, int64_t steps, int64_t streams,
                        int64_t step_stride, int64_t stream_stride, const int32_t *syms, int prec,
                        uint8_t *out, uint64_t cap_bytes, uint64_t *nbits, int32_t *status, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > streams) nthreads = (int)(streams > 0 ? streams : 1);
    pthread_t th[256];
    batch_arg args[256];
    if (nthreads > 256) nthreads = 256;
    for (int i = 0; i < nthreads; i++) {
        args[i] = (batch_arg){pmf, elem_bytes, V, steps, streams, step_stride, stream_stride, syms, prec,
                              out, cap_bytes, nbits, status, streams * i / nthreads, streams * (i + 1) / nthreads};
        pthread_create(&th[i], NULL, batch_worker, &args[i]);
    }
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    for (int64_t b = 0; b < streams; b++)
        if (status[b]) return status[b];
    return R_OK;
}

/* ---- value-register decoder == A_from_bin.run(bits,0)[:n] ---- */
static inline int getbit(const uint8_t *bytes, uint64_t nbits, uint64_t i) {
    return i < nbits ? (bytes[i >> 3] >> (7 - (i & 7))) & 1 : 0;
}

int lacref_decode(const void *pmf, int elem_bytes, int64_t V, int64_t nsym, int64_t step_stride,
                  const uint8_t *bytes, uint64_t nbits, int prec, int32_t *syms_out) {
    int rc = check_prec(prec, V);
    if (rc) return rc;
    const int64_t P = prec, D = (int64_t)1 << P, Hd = (int64_t)1 << (P - 1);
    uint64_t *cdf = malloc(sizeof(uint64_t) * V), *scr = malloc(sizeof(uint64_t) * V);
    if (!cdf || !scr) { free(cdf); free(scr); return R_E_ARG; }
    int64_t x = 0, l = 0, h = D - 1;
    uint64_t pos = 0;
    for (; pos < (uint64_t)P; pos++) x = (x << 1) | getbit(bytes, nbits, pos);
    for (int64_t t = 0; t < nsym; t++) {
        const void *row = (const char *)pmf + (size_t)(t * step_stride) * elem_bytes;
        uint64_t minp;
        if ((rc = build_cdf(row, elem_bytes, V, cdf, &minp))) break;
        uint64_t w = (uint64_t)(h - l + 1);
        const uint64_t *dist = fudged_dist(cdf, minp, V, w, scr);
        int64_t s = val_to_symbol(dist, V, (uint64_t)(x - l), w);
        uint64_t a, b;
        if ((rc = symbol_to_range(dist, V, s, w, &a, &b))) break;
        if (!(l + (int64_t)a <= x && x <= l + (int64_t)b - 1)) { rc = R_E_DECODE_RANGE; break; }
        h = l + (int64_t)b - 1;
        l += (int64_t)a;
        syms_out[t] = (int32_t)s;
        while (h - l < Hd) {
            int64_t d = l / Hd;
            l = l * 2 - d * D;
            h = h * 2 + 1 - d * D;
            x = x * 2 + getbit(bytes, nbits, pos++) - d * D;
        }
    }
    free(cdf); free(scr);
    return rc;
}

/* A_from_bin.run(bits, stop=0) literally (arith_code.py:264-299, :322-326): per
 * bit receive_bit halves [lb, hb]; while val_to_symbol of both window ends agree,
 * emit_symbol (with its overlap check) and the emit_bit loop over l, h, lb, hb.
 * Rows: step t uses row min(t, nrows-1).  Returns how many symbols the bits
 * determine, at most max_out (or a negative status). */
int64_t lacref_decode_bitserial(const void *pmf, int elem_bytes, int64_t V, int64_t nrows, int64_t step_stride,
                                const uint8_t *bytes, uint64_t nbits, int prec, int32_t *syms_out,
                                int64_t max_out) {
    int rc = check_prec(prec, V);
    if (rc) return rc;
    const int64_t D = (int64_t)1 << prec, Hd = (int64_t)1 << (prec - 1);
    uint64_t *cdf = malloc(sizeof(uint64_t) * V), *scr = malloc(sizeof(uint64_t) * V);
    if (!cdf || !scr) { free(cdf); free(scr); return R_E_ARG; }
    int64_t l = 0, h = D - 1, lb = 0, hb = D - 1, n = 0, row_of = -1;
    uint64_t minp = 0;
    for (uint64_t i = 0; i < nbits && rc == R_OK; i++) {
        const int64_t half = (hb - lb + 1) / 2;
        lb += half * getbit(bytes, nbits, i);
        hb = lb + half - 1;
        for (;;) {
            const int64_t r = n < nrows ? n : nrows - 1;
            if (r != row_of) {
                if ((rc = build_cdf((const char *)pmf + (size_t)(r * step_stride) * elem_bytes, elem_bytes, V, cdf,
                                    &minp)))
                    break;
                row_of = r;
            }
            const uint64_t w = (uint64_t)(h - l + 1);
            const uint64_t *dist = fudged_dist(cdf, minp, V, w, scr);
            /* lb >= l always holds here (a symbol is emitted only inside its range) */
            const int64_t ls = val_to_symbol(dist, V, (uint64_t)(lb - l), w);
            const int64_t hs = (hb - l) >= (int64_t)w ? V : val_to_symbol(dist, V, (uint64_t)(hb - l), w);
            if (ls != hs) break;
            uint64_t a, b;
            if ((rc = symbol_to_range(dist, V, ls, w, &a, &b))) break;
            if (region_overlap(l + (int64_t)a, l + (int64_t)b - 1, lb, hb) == 0) { rc = R_E_DECODE_RANGE; break; }
            h = l + (int64_t)b - 1;
            l += (int64_t)a;
            if (n >= max_out) break;      /* a one-symbol row determines symbols forever (the reference loops) */
            syms_out[n++] = (int32_t)ls;
            while (h - l < Hd) {
                const int64_t d = floordiv(l, Hd);
                l = l * 2 - d * D;
                h = h * 2 + 1 - d * D;
                lb = lb * 2 - d * D;
                hb = hb * 2 + 1 - d * D;
            }
        }
    }
    free(cdf); free(scr);
    return rc ? rc : n;
}

/* ---- ACSampler encode on a fixed uint64 CDF (arithmetic_coding.py) ---- */
int lacref_acsampler_encode(const uint64_t *cdf, int64_t V, const int32_t *toks, int64_t n, int prec,
                            uint8_t *bits_out, uint64_t cap_bits, uint64_t *nbits) {
    if (prec < 2 || prec > 62 || V < 1) return R_E_PREC;
    const i128 one = (i128)1 << prec;
    i128 low = 0, high = one - 1;
    u128 buf = 0;
    int64_t nbuf = 0;
    uint64_t L = 0;
    const u128 denom = cdf[V - 1];
#define ACS_OUT(bit)                                                   \
    do {                                                               \
        if (L >= cap_bits) return R_E_CAPACITY;                        \
        bits_out[L++] = (uint8_t)(bit);                                \
    } while (0)
#define ACS_FLUSH()                                                    \
    while (nbuf > 0) {                                                 \
        nbuf -= 1;                                                     \
        u128 b_ = buf >> nbuf;                                         \
        ACS_OUT(b_);                                                   \
        buf &= (((u128)1) << nbuf) - 1;                                \
    }
    for (int64_t i = 0; i <= n; i++) {
        u128 lo, hi, d;
        if (i < n) {                                           /* sample_scaled_cdf :86-90 */
            int64_t tok = toks[i];
            if (tok < 0 || tok >= V) return R_E_SYMBOL_RANGE;
            lo = tok ? cdf[tok - 1] : 0; hi = cdf[tok]; d = denom;
        } else {                                               /* flush_compress :50-56 */
            lo = 1; hi = 2; d = 3;
        }
        i128 span = high - low + 1;                            /* Region.step/map :160-168 */
        i128 nl = low + (i128)(((u128)span * lo) / d);
        i128 nh = low + (i128)(((u128)span * hi) / d) - 1;
        low = nl; high = nh;
        while ((high - low + 1) * 2 <= one) {                  /* Region.emit :169-174 */
            i128 bit = low >> (prec - 1);
            low = (low << 1) - (bit << prec);
            high = ((high << 1) + 1) - (bit << prec);
            if (nbuf >= 120) return R_E_CAPACITY;
            buf = (buf << 1) + (u128)bit;                      /* CarryBuffer.add :198-202 */
            nbuf += 1;
            if (high < one) { ACS_FLUSH(); }                   /* Region.definite :175-177 */
        }
    }
    ACS_FLUSH();
    *nbits = L;
    return R_OK;
#undef ACS_OUT
#undef ACS_FLUSH
}

/* ---- q1 logits quantiser (DESIGN.md "logits path"): bf16 (type 1) or f32 (type 2)
 * logits -> uint32 pmf.  With L = DMAX*STEPS = 544:
 *   m = max_i x_i (fmaxf: NaN ignored),  c = RNE_f32(L - 32 m),
 *   y = fmaf(x, 32, c) (one rounding),  j = 0 if y is NaN or y <= 0, else min(trunc(y), L),
 *   q = max(1, TAB[L - j] >> (24 - k)),  TAB[i] = round(2^24 e^(-i/32)),
 *   k = min(24, prec-1-ceil(log2 V)).
 * i = L - j is the logit gap m - x in 1/32-nat steps (rounded up), clamped at 17 nats. */
static inline float q1_load(const void *x, int type, int64_t i) {
    if (type == 1) {
        uint32_t u = (uint32_t)((const uint16_t *)x)[i] << 16;
        float f;
        memcpy(&f, &u, 4);
        return f;
    }
    return ((const float *)x)[i];
}

int lacref_q1_k(int prec, int64_t V) {
    int cl = 0;
    while (((int64_t)1 << cl) < V) cl++;
    int k = prec - 1 - cl;
    if (k > LAC_Q1_KMAX) k = LAC_Q1_KMAX;
    return k;
}

int lacref_q1_quantize(const void *x, int type, int64_t V, int prec, uint32_t *q) {
    const int k = lacref_q1_k(prec, V);
    if (k < 1 || (type != 1 && type != 2)) return R_E_ARG;
    float m = -INFINITY;
    for (int64_t i = 0; i < V; i++) m = fmaxf(m, q1_load(x, type, i));
    const int L = LAC_Q1_DMAX * LAC_Q1_STEPS;
    volatile float m32 = (float)LAC_Q1_STEPS * m;                     /* exact (power of two) */
    volatile float c = (float)L - m32;                                 /* one f32 rounding */
    for (int64_t i = 0; i < V; i++) {
        const float y = fmaf(q1_load(x, type, i), (float)LAC_Q1_STEPS, c);
        uint32_t j;
        if (!(y > 0.0f)) j = 0;                                         /* NaN, -inf, negative, zero */
        else if (y >= (float)L) j = (uint32_t)L;
        else j = (uint32_t)y;                                           /* truncation */
        uint32_t v = Q1_TAB[L - j] >> (LAC_Q1_KMAX - k);
        q[i] = v ? v : 1u;
    }
    return R_OK;
}
