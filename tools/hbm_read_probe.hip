// hbm_read_probe.hip -- achievable HBM read bandwidth on this MI355X, for context
// on the coder's roofline fraction (a measured ceiling, not the 8 TB/s spec).
//
//   hipcc --offload-arch=gfx950 -O3 tools/hbm_read_probe.hip -o tools/hbm_read_probe
//   tools/hbm_read_probe [GiB]
//
// Variants (all sum u32 words so no load is dead; 8 GiB buffer >> 256 MiB MALL):
//   gridstride<U,NT>  classic grid-stride stream, U x 16-B loads in flight per lane
//   rowwave<U,NT>     the coder's shape: one wave per 128 KiB row, rows in order
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__device__ inline u32x4 ld(const u32x4 *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void gridstride(const u32x4 *__restrict__ in, size_t n, uint32_t *out) {
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (size_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    size_t i = tid;
    for (; i + (U - 1) * nt < n; i += U * nt) {
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; u++) x[u] = ld<U, NT>(in + i + u * nt);
#pragma unroll
        for (int u = 0; u < U; u++) acc += x[u].x ^ x[u].y ^ x[u].z ^ x[u].w;
    }
    for (; i < n; i += nt) { u32x4 x = ld<U, NT>(in + i); acc += x.x ^ x.y ^ x.z ^ x.w; }
    if (acc == 0x12345678u) out[0] = acc;
}

// one wave per row of `rowvec` 16-B vectors, `rows` rows, each wave walks `per` rows
template <int U, bool NT>
__global__ __launch_bounds__(256) void rowwave(const u32x4 *__restrict__ in, size_t rowvec, size_t rows, size_t per,
                                               uint32_t *out) {
    const int lane = threadIdx.x & 63;
    const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    uint32_t acc = 0;
    for (size_t k = 0; k < per; k++) {
        const size_t r = w + k * ((size_t)gridDim.x * 4);
        if (r >= rows) break;
        const u32x4 *row = in + r * rowvec;
        size_t v = lane;
        for (; v + 64 * (U - 1) < rowvec; v += 64 * U) {
            u32x4 x[U];
#pragma unroll
            for (int u = 0; u < U; u++) x[u] = ld<U, NT>(row + v + 64 * u);
#pragma unroll
            for (int u = 0; u < U; u++) acc += x[u].x ^ x[u].y ^ x[u].z ^ x[u].w;
        }
        for (; v < rowvec; v += 64) { u32x4 x = ld<U, NT>(row + v); acc += x.x ^ x.y ^ x.z ^ x.w; }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <typename F>
static double time_ms(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; i++) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char **argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 8.0;
    const size_t bytes = (size_t)(gib * (1ull << 30)) / (128 * 1024) * (128 * 1024);
    const size_t n = bytes / 16;
    u32x4 *buf;
    uint32_t *out;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, 4));
    CK(hipMemset(buf, 0x5a, bytes));
    const int reps = 10;
    auto report = [&](const char *name, double ms) {
        printf("%-28s %8.3f ms  %7.1f GB/s  (%.1f %% of 8 TB/s)\n", name, ms, bytes / (ms * 1e-3) / 1e9,
               100.0 * bytes / (ms * 1e-3) / 8e12);
    };
#define GS(U, NT, BLK)                                                                                   \
    report("gridstride U=" #U " nt=" #NT " blk/CU=" #BLK,                                                 \
           time_ms([&] { gridstride<U, NT><<<256 * BLK, 256>>>(buf, n, out); }, reps))
    GS(4, true, 8); GS(8, true, 8); GS(8, false, 8); GS(16, true, 4); GS(8, true, 4); GS(8, true, 16);
    const size_t rowvec = 8000, rows = bytes / (rowvec * 16);   // 128,000-B rows (V = 32000 u32)
#define RW(U, NT, WAVES)                                                                                 \
    report("rowwave U=" #U " nt=" #NT " waves=" #WAVES,                                                   \
           time_ms([&] { rowwave<U, NT><<<(WAVES) / 4, 256>>>(buf, rowvec, rows, (rows + (WAVES) - 1) / (WAVES), out); }, reps))
    RW(8, true, 4096); RW(8, false, 4096); RW(8, true, 8192); RW(4, true, 4096); RW(16, true, 4096);
    RW(8, true, 2048); RW(8, true, 16384);
    CK(hipFree(buf));
    return 0;
}
