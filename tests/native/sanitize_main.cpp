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
