// rcp_probe.hip -- measure, on the MI355X, the error of the device reciprocal
// (v_rcp_f64, lac_core.h recip) against the correctly rounded 1/d, and the final
// +-1 corrections div_floor_inv needs with it; every quotient is checked against
// an exact 128-bit division.  Evidence for tests/test_core_host.py's bound.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I lac_amd/csrc tools/rcp_probe.hip -o tools/rcp_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include "lac_core.h"

using namespace lac;

__device__ inline uint64_t mix(uint64_t x) {           // splitmix64
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ void probe(uint64_t n, unsigned long long *max_ulp, unsigned long long *max_fix,
                      unsigned long long *bad) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t r0 = mix(i), r1 = mix(r0), r2 = mix(r1), r3 = mix(r2);
    const int dbits = 1 + (int)(r0 % 64);
    uint64_t d = r1 >> (64 - dbits);
    if (d == 0) d = 1;
    const double rc = recip(d), ie = 1.0 / (double)d;
    uint64_t a, b;
    memcpy(&a, &rc, 8);
    memcpy(&b, &ie, 8);
    const unsigned long long ulp = a > b ? a - b : b - a;
    atomicMax(max_ulp, ulp);
    // quotients up to 2^64 - 1
    const int qbits = 1 + (int)(r2 % 64);
    const uint64_t q = r3 >> (64 - qbits);
    const uint64_t rem = mix(r3) % d;
    const u128 N = (u128)q * d + rem;
    int fix = 0;
    const uint64_t got = div_floor_inv_n(N, d, rc, &fix);
    atomicMax(max_fix, (unsigned long long)fix);
    if (got != (uint64_t)(N / d)) atomicAdd(bad, 1ull);
}

int main() {
    unsigned long long *dv;
    hipMalloc(&dv, 3 * sizeof(unsigned long long));
    hipMemset(dv, 0, 3 * sizeof(unsigned long long));
    const uint64_t n = 1ull << 24;
    probe<<<(unsigned)(n / 256), 256>>>(n, dv, dv + 1, dv + 2);
    unsigned long long h[3];
    hipMemcpy(h, dv, sizeof h, hipMemcpyDeviceToHost);
    printf("{\"cases\": %llu, \"max_rcp_ulp_vs_ieee\": %llu, \"max_fixups\": %llu, \"wrong_quotients\": %llu}\n",
           (unsigned long long)n, h[0], h[1], h[2]);
    return h[2] != 0;
}
