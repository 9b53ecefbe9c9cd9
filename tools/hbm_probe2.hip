// hbm_probe2.hip -- round-2 HBM read-ceiling sweep on MI355X: which load shape and
// cache policy streams 128 KB rows fastest (the coder's access pattern).
//
//   hipcc --offload-arch=gfx950 -O3 tools/hbm_probe2.hip -o tools/hbm_probe2
//   tools/hbm_probe2 [GiB]
//
// Every variant sums the u32 words it reads (no dead loads); the buffer is
// 8 GiB >> the 256 MiB MALL.  Variants:
//   row<U,AUX>   one wave per 128,000-B row, U x 16-B buffer loads in flight per
//                lane, cache-policy bits AUX (gfx950: 1 = sc0, 2 = nt, 16 = sc1)
//   wgrow<U,AUX> one 4-wave workgroup per row (each instruction covers 4 KB)
//   glob<U>      the round-1 shape: global_load with __builtin_nontemporal_load
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int AUX>
__device__ inline u32x4 bld(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX);
}

__device__ inline uint32_t fold(u32x4 x) { return x.x ^ x.y ^ x.z ^ x.w; }

// one wave per row; rows visited w, w + nwaves, ...
template <int U, int AUX>
__global__ __launch_bounds__(256) void row(const u32x4 *__restrict__ in, uint32_t rowvec, size_t rows,
                                           uint32_t *out) {
    const int lane = threadIdx.x & 63;
    const size_t nw = (size_t)gridDim.x * 4;
    uint32_t acc = 0;
    for (size_t r = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += nw) {
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(in + r * rowvec), 0, rowvec * 16,
                                                                      0x00020000);
        uint32_t v = lane;
        for (; v + 64 * (U - 1) < rowvec; v += 64 * U) {
            u32x4 x[U];
#pragma unroll
            for (int u = 0; u < U; u++) x[u] = bld<AUX>(rs, (v + 64 * u) * 16);
#pragma unroll
            for (int u = 0; u < U; u++) acc += fold(x[u]);
        }
        for (; v < rowvec; v += 64) acc += fold(bld<AUX>(rs, v * 16));
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// one 4-wave workgroup per row
template <int U, int AUX>
__global__ __launch_bounds__(256) void wgrow(const u32x4 *__restrict__ in, uint32_t rowvec, size_t rows,
                                             uint32_t *out) {
    const int t = threadIdx.x;
    uint32_t acc = 0;
    for (size_t r = blockIdx.x; r < rows; r += gridDim.x) {
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(in + r * rowvec), 0, rowvec * 16,
                                                                      0x00020000);
        uint32_t v = t;
        for (; v + 256 * (U - 1) < rowvec; v += 256 * U) {
            u32x4 x[U];
#pragma unroll
            for (int u = 0; u < U; u++) x[u] = bld<AUX>(rs, (v + 256 * u) * 16);
#pragma unroll
            for (int u = 0; u < U; u++) acc += fold(x[u]);
        }
        for (; v < rowvec; v += 256) acc += fold(bld<AUX>(rs, v * 16));
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int U>
__global__ __launch_bounds__(256) void glob(const u32x4 *__restrict__ in, uint32_t rowvec, size_t rows,
                                            uint32_t *out) {
    const int lane = threadIdx.x & 63;
    const size_t nw = (size_t)gridDim.x * 4;
    uint32_t acc = 0;
    for (size_t r = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += nw) {
        const u32x4 *p = in + r * rowvec;
        uint32_t v = lane;
        for (; v + 64 * (U - 1) < rowvec; v += 64 * U) {
            u32x4 x[U];
#pragma unroll
            for (int u = 0; u < U; u++) x[u] = __builtin_nontemporal_load(p + v + 64 * u);
#pragma unroll
            for (int u = 0; u < U; u++) acc += fold(x[u]);
        }
        for (; v < rowvec; v += 64) acc += fold(__builtin_nontemporal_load(p + v));
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
    const uint32_t rowvec = 8000;                                   // 128,000-B rows (V = 32000 u32)
    const size_t rows = (size_t)(gib * (1ull << 30)) / (rowvec * 16);
    const size_t bytes = rows * rowvec * 16;
    u32x4 *buf;
    uint32_t *out;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, 4));
    CK(hipMemset(buf, 0x5a, bytes));
    const int reps = 10;
    auto report = [&](const char *name, double ms) {
        printf("%-34s %8.3f ms  %7.1f GB/s  (%.1f %% of 8 TB/s)\n", name, ms, bytes / (ms * 1e-3) / 1e9,
               100.0 * bytes / (ms * 1e-3) / 8e12);
        fflush(stdout);
    };
#define ROW(U, AUX, W) report("row U=" #U " aux=" #AUX " waves=" #W, \
        time_ms([&] { row<U, AUX><<<(W) / 4, 256>>>(buf, rowvec, rows, out); }, reps))
#define WG(U, AUX, G) report("wgrow U=" #U " aux=" #AUX " wgs=" #G, \
        time_ms([&] { wgrow<U, AUX><<<(G), 256>>>(buf, rowvec, rows, out); }, reps))
#define GL(U, W) report("glob U=" #U " waves=" #W, \
        time_ms([&] { glob<U><<<(W) / 4, 256>>>(buf, rowvec, rows, out); }, reps))
    GL(8, 2048); GL(8, 4096);
    ROW(8, 2, 2048); ROW(8, 2, 4096);
    ROW(8, 0, 2048); ROW(8, 1, 2048); ROW(8, 3, 2048); ROW(8, 16, 2048); ROW(8, 17, 2048); ROW(8, 18, 2048);
    ROW(8, 19, 2048);
    ROW(12, 2, 2048); ROW(16, 2, 2048); ROW(16, 2, 1024); ROW(8, 2, 1024); ROW(4, 2, 4096); ROW(4, 2, 8192);
    ROW(8, 18, 4096); ROW(16, 18, 2048);
    WG(4, 2, 512); WG(4, 2, 1024); WG(8, 2, 512); WG(8, 2, 1024); WG(2, 2, 2048); WG(4, 18, 1024);
    GL(8, 2048);
    CK(hipFree(buf));
    return 0;
}
