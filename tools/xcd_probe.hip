// Where the workgroups of one launch run: XCC (XCD) id and HW_ID (SE / CU / SIMD) of each
// workgroup of a 64-thread launch, workgroup 0 spinning ~2 ms as the lean decoder does
// (tools/sessions/gpu_r06_s.sh).  Checks the layout k_decode_lean assumes: workgroup j on
// XCD (j mod 8) relative to workgroup 0.
//   hipcc --offload-arch=gfx950 -O2 tools/xcd_probe.hip -o tools/_probe/xcd_probe && tools/_probe/xcd_probe 648
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void k_where(unsigned *out, long long spin) {
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);   // HW_REG_XCC_ID[3:0]
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    if (blockIdx.x == 0) {
        const long long t0 = clock64();
        while (clock64() - t0 < spin) __builtin_amdgcn_s_sleep(1);
    }
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = xcc;
        out[2 * blockIdx.x + 1] = hw;
    }
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 648;
    unsigned *d, *h = (unsigned *)malloc(sizeof(unsigned) * 2 * n);
    if (hipMalloc(&d, sizeof(unsigned) * 2 * n) != hipSuccess) return 1;
    for (int rep = 0; rep < 3; rep++) {
        k_where<<<n, 64>>>(d, 4000000LL);
        if (hipMemcpy(h, d, sizeof(unsigned) * 2 * n, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        int agree = 0;
        const unsigned x0 = h[0];
        for (int j = 0; j < n; j++) agree += (h[2 * j] == ((x0 + j) & 7));
        printf("rep %d: workgroup 0 on XCC %u; workgroups on XCC (x0 + j) mod 8: %d of %d\n", rep, x0, agree, n);
        const unsigned cu0 = (h[1] >> 8) & 15, se0 = (h[1] >> 13) & 7, simd0 = (h[1] >> 4) & 3;
        int same_cu = 0, same_xcc = 0;
        for (int j = 1; j < n; j++) {
            if (h[2 * j] == x0) {
                same_xcc++;
                if (((h[2 * j + 1] >> 8) & 15) == cu0 && ((h[2 * j + 1] >> 13) & 7) == se0) same_cu++;
            }
        }
        printf("  workgroup 0: SE %u CU %u SIMD %u; others on its XCC: %d, on its CU: %d\n", se0, cu0, simd0, same_xcc,
               same_cu);
        if (rep == 0) {
            printf("  first 24 (xcc:se:cu):");
            for (int j = 0; j < 24 && j < n; j++)
                printf(" %u:%u:%u", h[2 * j], (h[2 * j + 1] >> 13) & 7, (h[2 * j + 1] >> 8) & 15);
            printf("\n");
        }
    }
    return 0;
}
