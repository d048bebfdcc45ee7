// Where do the two waves of a 128-thread workgroup run?  Each wave records
// HW_ID (gfx9 layout: wave [3:0], SIMD [5:4], CU [11:8], SH [12], SE [15:13])
// while it holds the same LDS and register footprint as k_qp_tiled2.
// Build: hipcc --offload-arch=gfx950 -O3 -o simd_place simd_place.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <map>

__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_place(unsigned* out, double* sink) {
    extern __shared__ double lds[];
    const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 2 + (threadIdx.x >> 6)] = hw;
    double v = threadIdx.x;
    for (int k = 0; k < 20000; ++k) v = fma(v, 1.0000001, 1e-9);   // hold the slot a while
    lds[threadIdx.x] = v;
    __syncthreads();
    if (v == 1.2345) sink[blockIdx.x] = lds[127 - threadIdx.x];
}

int main() {
    const int B = 4096;
    unsigned* d; double* s;
    hipMalloc(&d, B * 2 * sizeof(unsigned)); hipMalloc(&s, B * sizeof(double));
    hipLaunchKernelGGL(k_place, dim3(B), dim3(128), 37520, 0, d, s);
    hipDeviceSynchronize();
    unsigned* h = (unsigned*)malloc(B * 2 * sizeof(unsigned));
    hipMemcpy(h, d, B * 2 * sizeof(unsigned), hipMemcpyDeviceToHost);
    int same_simd = 0, same_cu = 0;
    std::map<int, int> simd_pairs;
    for (int b = 0; b < B; ++b) {
        const unsigned a = h[2 * b], c = h[2 * b + 1];
        const unsigned cua = (a >> 8) & 0xF, cuc = (c >> 8) & 0xF, sa = (a >> 4) & 3, sc = (c >> 4) & 3;
        const unsigned sea = (a >> 13) & 7, sec = (c >> 13) & 7, sha = (a >> 12) & 1, shc = (c >> 12) & 1;
        const bool cu = cua == cuc && sea == sec && sha == shc;
        same_cu += cu;
        same_simd += cu && sa == sc;
        simd_pairs[sa * 4 + sc]++;
    }
    printf("blocks %d: both waves on one CU %d, on one SIMD %d\n", B, same_cu, same_simd);
    for (auto& kv : simd_pairs) printf("  simd(wave0)=%d simd(wave1)=%d : %d\n", kv.first / 4, kv.first % 4, kv.second);
    for (int b = 0; b < 8; ++b) printf("  block %d: %08x %08x\n", b, h[2 * b], h[2 * b + 1]);
    return 0;
}
