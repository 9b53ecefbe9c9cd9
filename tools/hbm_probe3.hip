// hbm_probe3.hip -- round-3 HBM read-ceiling probe on MI355X: do deeper queues of
// LDS-DMA loads (global_load_lds_dwordx4: no VGPRs held per load) read faster than
// round 2's best register shape (row U=8 nt, 2 waves/SIMD: 7.03 TB/s, hbm_probe2)?
//
//   hipcc --offload-arch=gfx950 -O3 tools/hbm_probe3.hip -o tools/hbm_probe3
//   tools/hbm_probe3 [GiB]
//
// dma<U, WPB, NT>: blocks of WPB waves, one wave per 128,000-B row (as the coder's
// streams), each wave keeps U/2..U 1-KB DMA loads in flight into its own U-KB LDS
// ring (rolling: wait until <= U/2 are outstanding, issue U/2 more); NT = the nt
// cache-policy bit.  The data lands in LDS and is not read (the asm loads cannot
// be elided).  Register shapes from hbm_probe2 are repeated as the reference.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lvoid_t;

template <int N>
constexpr int vmcnt_imm() {                       // s_waitcnt vmcnt(N), no lgkm / exp wait (gfx9 encoding)
    return (N & 15) | (7 << 4) | (15 << 8) | (((N >> 4) & 3) << 14);
}

template <bool NT>
__device__ inline void dma16(const u32x4 *src, uint32_t lds_addr) {
    const uint32_t lds = __builtin_amdgcn_readfirstlane(lds_addr);   // m0 takes an SGPR
    uint32_t keep;
    if constexpr (NT)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
}

template <int U, int WPB, bool NT>
__global__ __launch_bounds__(64 * WPB) void dma(const u32x4 *__restrict__ in, uint32_t rowvec, size_t rows,
                                                uint32_t *out) {
    constexpr int H = U / 2;
    __shared__ u32x4 ring[WPB * U * 64];
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint32_t base = (uint32_t)(uintptr_t)(lvoid_t *)&ring[w * U * 64];
    const size_t nw = (size_t)gridDim.x * WPB;
    int slot = 0;
    for (size_t r = (size_t)blockIdx.x * WPB + w; r < rows; r += nw) {
        const u32x4 *p = in + r * rowvec;
        uint32_t v = lane;
        for (; v + 64 * (H - 1) < rowvec; v += 64 * H) {
            __builtin_amdgcn_s_waitcnt(vmcnt_imm<H>());
#pragma unroll
            for (int u = 0; u < H; u++) dma16<NT>(p + v + 64 * u, base + (uint32_t)(((slot + u) % U) * 1024));
            slot = (slot + H) % U;
        }
        for (; v < rowvec; v += 64) {
            __builtin_amdgcn_s_waitcnt(vmcnt_imm<H>());
            dma16<NT>(p + v, base + (uint32_t)(slot * 1024));
            slot = (slot + 1) % U;
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    if (lane == 0 && w == 0 && rows == 0) out[0] = 1;
}

template <int AUX>
__device__ inline u32x4 bld(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX);
}
__device__ inline uint32_t fold(u32x4 x) { return x.x ^ x.y ^ x.z ^ x.w; }

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
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    u32x4 *buf;
    uint32_t *out;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, 4));
    CK(hipMemset(buf, 0x5a, bytes));
    const int reps = 10;
    auto report = [&](const char *name, double ms) {
        printf("%-40s %8.3f ms  %7.1f GB/s  (%.1f %% of 8 TB/s)\n", name, ms, bytes / (ms * 1e-3) / 1e9,
               100.0 * bytes / (ms * 1e-3) / 8e12);
        fflush(stdout);
    };
#define ROW(U, AUX, W) report("row U=" #U " aux=" #AUX " waves=" #W, \
        time_ms([&] { row<U, AUX><<<(W) / 4, 256>>>(buf, rowvec, rows, out); }, reps))
    // DMA(U KB per wave, WPB waves per block, BPC blocks per CU, NT)
#define DMA(U, WPB, BPC, NT) report("dma U=" #U "KB wpb=" #WPB " bpc=" #BPC " nt=" #NT, \
        time_ms([&] { dma<U, WPB, NT><<<cus * (BPC), 64 * (WPB)>>>(buf, rowvec, rows, out); }, reps))
    ROW(8, 2, 2048);
    DMA(8, 4, 2, false); DMA(16, 4, 2, false); DMA(32, 4, 1, false);
    DMA(8, 8, 2, false); DMA(16, 8, 1, false); DMA(8, 16, 1, false);
    DMA(16, 4, 2, true); DMA(8, 16, 1, true); DMA(32, 4, 1, true);
    DMA(4, 16, 2, true); DMA(8, 8, 2, true); DMA(16, 8, 1, true);
    DMA(4, 8, 4, true); DMA(2, 16, 4, true);
    ROW(8, 2, 2048);
    CK(hipFree(buf));
    return 0;
}
