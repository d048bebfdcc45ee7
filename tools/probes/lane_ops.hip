// Probe of gfx950 cross-lane primitives: prints, for each lane, which source
// lane each op delivers (inputs are lane ids).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* o) {
    const int l = threadIdx.x;
    const int a = l, b = 100 + l;
    auto p32 = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    auto p16 = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    o[0 * 64 + l] = p32[0];
    o[1 * 64 + l] = p32[1];
    o[2 * 64 + l] = p16[0];
    o[3 * 64 + l] = p16[1];
    o[4 * 64 + l] = __builtin_amdgcn_update_dpp(-1, a, 0x153, 0xF, 0xF, false);   // row_newbcast:3
    o[5 * 64 + l] = __builtin_amdgcn_update_dpp(-1, a, 0x142, 0xF, 0xF, false);   // row_bcast:15
    o[6 * 64 + l] = __builtin_amdgcn_update_dpp(-1, a, 0x143, 0xF, 0xF, false);   // row_bcast:31
    o[7 * 64 + l] = __builtin_amdgcn_update_dpp(-1, a, 0x111, 0xF, 0xF, false);   // row_shr:1
}
int main() {
    int* d; hipMalloc(&d, 8 * 64 * sizeof(int));
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    int h[8 * 64]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char* names[] = {"p32.vdst", "p32.vsrc", "p16.vdst", "p16.vsrc", "newbcast3", "bcast15", "bcast31", "row_shr1"};
    for (int r = 0; r < 8; ++r) { printf("%-10s", names[r]); for (int l = 0; l < 64; ++l) printf(" %d", h[r * 64 + l]); printf("\n"); }
    return 0;
}
