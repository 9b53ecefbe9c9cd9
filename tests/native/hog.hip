// hog.hip -- test infrastructure: a kernel that holds CUs for a given time, so a
// test can run the coder while part of the GPU is taken by another kernel.
// One 1024-thread block per CU (96 KB of LDS each keeps a second hog block and
// any 160 KB row-group block off that CU); every block spins on the 100 MHz s_memrealtime clock until its
// deadline, with a hard poll bound so it always ends.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(1024) void k_hog(uint64_t ticks, uint32_t *done) {
    __shared__ uint32_t pad[24576];                      // 96 KB: one hog block per CU
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t n = 0;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks && n < (1u << 26)) {
        __builtin_amdgcn_s_sleep(10);
        n++;
    }
    pad[threadIdx.x] = n;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(done, pad[1023] > 0 ? 1u : 0u);
}

extern "C" int hog_launch(int blocks, double seconds, uint32_t *done_dev, void *stream) {
    k_hog<<<blocks, 1024, 0, (hipStream_t)stream>>>((uint64_t)(seconds * 1e8), done_dev);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
