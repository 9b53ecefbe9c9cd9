// sanitize_main.cpp -- test infrastructure: the host-side coder arithmetic
// (lac_core.h, through core_check.cpp) and the C oracle (oracle/lac_oracle.c)
// built together with AddressSanitizer + UndefinedBehaviorSanitizer
// (tests/native/Makefile, target `asan`) and cross-checked on seeded random
// inputs: exact 128-bit division (incl. an inexact reciprocal), Python-rounded
// ratios, whole encodes core vs oracle, oracle encode -> decode round trips.
// Exit status 0 = every check passed and no sanitizer report.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

typedef unsigned __int128 u128;

extern "C" {
uint64_t cc_div_floor(uint64_t nh, uint64_t nl, uint64_t d);
uint64_t cc_div_floor_inv_ulp(uint64_t nh, uint64_t nl, uint64_t d, int ulps, int *fixups);
uint64_t cc_frac_mul_div(uint64_t c, uint64_t w, uint64_t T, int ceil);
uint64_t cc_cr_ratio(uint64_t a, uint64_t b);
int cc_encode(const void *pmf, int eb, int64_t V, int64_t steps, int64_t step_stride, const int32_t *syms, int prec,
              uint8_t *out, uint64_t cap_bytes, uint64_t *nbits);
int lacref_encode(const void *pmf, int elem_bytes, int64_t V, int64_t steps, int64_t step_stride,
                  const int32_t *syms, int prec, uint8_t *out, uint64_t cap_bytes, uint64_t *nbits, int8_t *digits,
                  uint64_t cap_digits, uint64_t *ndigits, int64_t *fail_step);
int lacref_decode(const void *pmf, int elem_bytes, int64_t V, int64_t nsym, int64_t step_stride,
                  const uint8_t *bytes, uint64_t nbits, int prec, int32_t *syms_out);
int64_t lacref_decode_bitserial(const void *pmf, int elem_bytes, int64_t V, int64_t nrows, int64_t step_stride,
                                const uint8_t *bytes, uint64_t nbits, int prec, int32_t *syms_out, int64_t max_out);
int cc_hc_encode_symbol(int prec, int64_t *l, int64_t *h, int64_t lo, int64_t hi, int8_t *digits, int32_t *n);
int cc_hc_encode_flush(int prec, int64_t l, int64_t h, int8_t *digits, int32_t *n);
int cc_hc_decode_emit(int prec, int64_t *regs, int64_t lo, int64_t hi, int renormalise);
}

// ---- the reference's register arithmetic (arith_code.py:169-202, 274-291) in 128
// bits, with lac_hc.h's refusal rule (registers must stay within +-2^62), as the
// model the host functions are checked against
typedef __int128 i128;
static const i128 LIM = (i128)1 << 62;
static bool in_lim(i128 a, i128 b) { return a > -LIM && a < LIM && b > -LIM && b < LIM; }
static i128 fdiv(i128 a, i128 b) { i128 q = a / b; return (a % b != 0 && a < 0) ? q - 1 : q; }
static i128 ovl(i128 a, i128 b, i128 c, i128 d) { i128 r = (d < b ? d : b) - (a > c ? a : c) + 1; return r > 0 ? r : 0; }

static int m_encode_symbol(int prec, i128 &l, i128 &h, i128 lo, i128 hi, std::vector<int> &dig) {
    if (hi <= lo) return -4;
    if (!in_lim(l, h)) return -1;
    i128 L = l + lo, H = l + hi - 1;
    if (!in_lim(L, H)) return -1;
    const i128 D = (i128)1 << prec, Hd = D >> 1;
    while (H - L < Hd) {
        const i128 d = fdiv(L, Hd);
        if (dig.size() >= 64 || d < -128 || d > 127) return -1;
        dig.push_back((int)d);
        L = 2 * L - d * D;
        H = 2 * H + 1 - d * D;
        if (!in_lim(L, H)) return -1;
    }
    l = L, h = H;
    return 0;
}

static int m_encode_flush(int prec, i128 l, i128 h, std::vector<int> &dig) {
    if (!in_lim(l, h)) return -1;
    const i128 D = (i128)1 << prec, Hd = D >> 1;
    while (l > 0 || h + 1 < D) {
        i128 d = fdiv(l, Hd);
        if (ovl(l, h, d * Hd, (d + 1) * Hd) < ovl(l, h, (d + 1) * Hd, (d + 2) * Hd)) d += 1;
        if (dig.size() >= 64 || d < -128 || d > 127) return -1;
        dig.push_back((int)d);
        l = 2 * l - d * D;
        h = 2 * h + 1 - d * D;
        if (!in_lim(l, h)) return -1;
    }
    return 0;
}

static int m_decode_emit(int prec, i128 *r, i128 lo, i128 hi, int renorm) {
    if (!in_lim(r[0], r[1]) || !in_lim(r[2], r[3])) return -1;
    i128 l = r[0] + lo, h = r[0] + hi - 1, lb = r[2], hb = r[3];
    if (ovl(l, h, lb, hb) == 0) return -6;
    if (!in_lim(l, h)) return -1;
    const i128 D = (i128)1 << prec, Hd = D >> 1;
    int n = 0;
    while (renorm && h - l < Hd) {
        const i128 d = fdiv(l, Hd);
        l = 2 * l - d * D, h = 2 * h + 1 - d * D, lb = 2 * lb - d * D, hb = 2 * hb + 1 - d * D;
        if (++n > 128 || !in_lim(l, h) || !in_lim(lb, hb)) return -1;
    }
    r[0] = l, r[1] = h, r[2] = lb, r[3] = hb;
    return 0;
}

static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t rnd() {                                   // splitmix64
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static uint64_t below(uint64_t n) { return n ? rnd() % n : 0; }
static int fails = 0;
#define CHECK(c, ...) do { if (!(c)) { fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); if (++fails > 20) exit(1); } } while (0)

int main() {
    // exact floor division, also with the reciprocal 4 ULPs off
    for (int i = 0; i < 200000; i++) {
        const uint64_t d = 1 + (rnd() >> below(64));
        const uint64_t q = rnd() >> below(64), r = below(d);
        const u128 N = (u128)q * d + r;
        CHECK(cc_div_floor((uint64_t)(N >> 64), (uint64_t)N, d) == q, "div_floor");
        int fix = 0;
        const int ulps = (int)below(9) - 4;
        CHECK(cc_div_floor_inv_ulp((uint64_t)(N >> 64), (uint64_t)N, d, ulps, &fix) == q && fix <= 2, "div_floor_inv");
    }
    fprintf(stderr, "div ok\n");
    // ceil/floor through row fractions
    for (int i = 0; i < 200000; i++) {
        const uint64_t T = 1 + (rnd() >> (1 + below(63)));
        const uint64_t c = below(T + 1);
        const int prec = 2 + (int)below(60);
        const uint64_t w = ((uint64_t)1 << (prec - 1)) + 1 + below((uint64_t)1 << (prec - 1));
        const u128 p = (u128)c * w;
        const uint64_t fl = (uint64_t)(p / T), ce = (uint64_t)((p + T - 1) / T);
        if (T >> 63) continue;
        CHECK(cc_frac_mul_div(c, w, T, 0) == fl && cc_frac_mul_div(c, w, T, 1) == ce, "frac_mul_div");
    }
    fprintf(stderr, "frac ok\n");
    // predictor-mapped host register functions (lac_hc.h) at every prec up to 61,
    // registers up to +-2^62, ranges anywhere in int64: equal to the 128-bit model,
    // and (this build) free of signed overflow
    for (int i = 0; i < 300000; i++) {
        const int prec = 2 + (int)below(60);
        const int64_t D = (int64_t)1 << prec;
        auto reg = [&]() -> int64_t {
            switch (below(4)) {
            case 0: return (int64_t)below((uint64_t)2 * D);                     // a coder's own range
            case 1: return ((int64_t)1 << 62) - 1 - (int64_t)below(1 << 20);    // at the limit
            case 2: return -((int64_t)1 << 62) + 1 + (int64_t)below(1 << 20);
            default: return (int64_t)rnd();                                    // anything
            }
        };
        int64_t l = reg(), h = reg();
        if (below(3) && l < ((int64_t)1 << 62) - D) h = l + (int64_t)below((uint64_t)D);
        const i128 w128 = (i128)h - l + 1;
        const uint64_t w = w128 > 0 && w128 < ((i128)1 << 62) ? (uint64_t)w128 : 1;
        int64_t lo = below(4) ? (int64_t)below(w) : (int64_t)rnd();
        int64_t hi = below(4) && lo < ((int64_t)1 << 62) ? lo + 1 + (int64_t)below(w) : (int64_t)rnd();
        if (below(8) == 0) hi = lo;
        int64_t L = l, H = h;
        int8_t dg[64];
        int32_t nd = 0;
        const int rc = cc_hc_encode_symbol(prec, &L, &H, lo, hi, dg, &nd);
        i128 ml = l, mh = h;
        std::vector<int> md;
        const int mrc = m_encode_symbol(prec, ml, mh, lo, hi, md);
        CHECK(rc == mrc, "hc_encode_symbol rc %d vs %d (prec %d)", rc, mrc, prec);
        if (rc == 0 && mrc == 0) {
            CHECK(L == (int64_t)ml && H == (int64_t)mh && nd == (int)md.size(), "hc_encode_symbol registers");
            for (int k = 0; k < nd && k < (int)md.size(); k++) CHECK(dg[k] == md[k], "hc_encode_symbol digit");
        }
        nd = 0;
        const int rf = cc_hc_encode_flush(prec, l, h, dg, &nd);
        md.clear();
        const int mrf = m_encode_flush(prec, l, h, md);
        CHECK(rf == mrf && (rf || nd == (int)md.size()), "hc_encode_flush rc %d vs %d (prec %d)", rf, mrf, prec);
        for (int k = 0; rf == 0 && k < nd && k < (int)md.size(); k++) CHECK(dg[k] == md[k], "hc_encode_flush digit");
        int64_t r4[4] = {l, h, reg(), 0};
        r4[3] = below(2) && r4[2] < ((int64_t)1 << 62) - D ? r4[2] + (int64_t)below((uint64_t)D) : reg();
        i128 m4[4] = {r4[0], r4[1], r4[2], r4[3]};
        const int ren = (int)below(2);
        const int re = cc_hc_decode_emit(prec, r4, lo, hi, ren);
        const int mre = m_decode_emit(prec, m4, lo, hi, ren);
        CHECK(re == mre, "hc_decode_emit rc %d vs %d (prec %d)", re, mre, prec);
        if (re == 0 && mre == 0)
            for (int k = 0; k < 4; k++) CHECK(r4[k] == (int64_t)m4[k], "hc_decode_emit registers");
    }
    fprintf(stderr, "hc ok\n");
    // Python-rounded ratios: the double nearest a/b (checked by exact integer bounds)
    for (int i = 0; i < 200000; i++) {
        const uint64_t b = 1 + (rnd() >> (1 + below(63)));
        const uint64_t a = below(b + 1);
        const uint64_t bitsv = cc_cr_ratio(a, b);
        double r;
        memcpy(&r, &bitsv, 8);
        CHECK(r >= 0.0 && r <= 1.0, "cr_ratio range");
        if (a == 0 || a == b) { CHECK(r == (a ? 1.0 : 0.0), "cr_ratio ends"); continue; }
        // |r - a/b| <= half an ulp of r: with r = m 2^e, check |m 2^e b - a| * 2 <= 2^e b (scaled)
        int e;
        const double m = frexp(r, &e);                      // r = m 2^e, m in [0.5, 1)
        const uint64_t M = (uint64_t)ldexp(m, 53);           // r = M 2^(e-53)
        const int sh = 53 - e;                               // r = M / 2^sh, sh in [53, 128)
        if (sh >= 120) continue;
        const u128 lhs = (u128)M * b, rhs = (u128)a << (sh > 63 ? 63 : sh);
        if (sh > 63) continue;                               // (covered by the Python-side test)
        const u128 diff = lhs > rhs ? lhs - rhs : rhs - lhs; // = |r - a/b| * b * 2^sh
        CHECK(diff * 2 <= (u128)b, "cr_ratio rounding %llu / %llu", (unsigned long long)a, (unsigned long long)b);
    }
    fprintf(stderr, "ratio ok\n");
    // whole encodes: the kernels' host arithmetic (core) == the oracle; oracle round trips
    for (int it = 0; it < 3000; it++) {
        const int64_t V = 2 + (int64_t)below(300);
        int prec = 2;
        while (((int64_t)1 << (prec - 1)) < V) prec++;
        prec += (int)below((uint64_t)(62 - prec));
        const int64_t steps = 1 + (int64_t)below(60);
        const bool wide = below(2);
        const int eb = wide ? 8 : 4;
        std::vector<uint64_t> rows64((size_t)(steps * V));
        std::vector<uint32_t> rows32((size_t)(steps * V));
        std::vector<int32_t> syms((size_t)steps);
        for (int64_t t = 0; t < steps; t++) {
            for (int64_t i = 0; i < V; i++) {
                const uint64_t v = below(4) == 0 ? 0 : 1 + (rnd() >> (wide ? 8 + below(40) : 40 + below(24)));
                rows64[(size_t)(t * V + i)] = v;
                rows32[(size_t)(t * V + i)] = (uint32_t)v;
            }
            const int64_t si = (int64_t)below((uint64_t)V), other = (si + 1 + (int64_t)below((uint64_t)V - 1)) % V;
            for (int64_t k : {si, other})                     // >= 2 positive entries: a one-symbol row
                if ((wide ? rows64[(size_t)(t * V + k)] : rows32[(size_t)(t * V + k)]) == 0) {   // decodes forever
                    if (wide) rows64[(size_t)(t * V + k)] = 1; else rows32[(size_t)(t * V + k)] = 1;
                }
            syms[(size_t)t] = (int32_t)si;
        }
        const void *pmf = wide ? (const void *)rows64.data() : (const void *)rows32.data();
        const uint64_t cap = (uint64_t)(steps * (prec + 2) + 128) / 8 + 16;
        std::vector<uint8_t> a(cap + 8), b(cap + 8);
        std::vector<int8_t> dg((size_t)(steps * (prec + 2) + 64));
        uint64_t na = 0, nb = 0, nd = 0;
        int64_t es = -1;
        const int ra = cc_encode(pmf, eb, V, steps, V, syms.data(), prec, a.data(), cap / 8 * 8, &na);
        const int rb = lacref_encode(pmf, eb, V, steps, V, syms.data(), prec, b.data(), cap, &nb, dg.data(), dg.size(),
                                     &nd, &es);
        CHECK(ra == rb, "encode status %d vs %d (V %lld prec %d)", ra, rb, (long long)V, prec);
        if (ra || rb) continue;
        CHECK(na == nb && memcmp(a.data(), b.data(), (size_t)((na + 7) / 8)) == 0, "encode bytes");
        std::vector<int32_t> out((size_t)steps + 64);
        CHECK(lacref_decode(pmf, eb, V, steps, V, b.data(), nb, prec, out.data()) == 0 &&
                  memcmp(out.data(), syms.data(), (size_t)steps * 4) == 0, "decode");
        const int64_t n = lacref_decode_bitserial(pmf, eb, V, steps, V, b.data(), nb, prec, out.data(), steps + 64);
        CHECK(n >= steps && memcmp(out.data(), syms.data(), (size_t)steps * 4) == 0, "bit-serial decode");
    }
    printf("sanitize_main: %s\n", fails ? "FAILED" : "ok");
    return fails ? 1 : 0;
}
