// Probe (tools only): read bandwidth of the [A_k | B_k] access pattern of
// k_expand20 / k_condense20 -- lane p of a 16-lane row reads row p's 128 bytes
// as 8 dwordx4 loads (128-byte stride across lanes) -- against a fully
// coalesced dwordx4 stream over the same bytes, and the same pattern with
// 2 waves per SIMD.  hipcc --offload-arch=gfx950 -O3 -o /tmp/rsb row_stride_bw.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef double double2v __attribute__((ext_vector_type(2)));

// rows of 16 doubles; wave handles 4 blocks of 13 rows per "interval", 20 intervals
__global__ __launch_bounds__(64) void k_rows(const double* __restrict__ a, double* __restrict__ out, int nwaves) {
    const int w = blockIdx.x, l = threadIdx.x, g = l >> 4, p = min(l & 15, 12);
    if (w >= nwaves) return;
    double acc = 0.0;
    for (int k = 0; k < 20; ++k) {
        const double2v* src = reinterpret_cast<const double2v*>(a + (((size_t)(4 * w + g) * 20 + k) * 13 + p) * 16);
        double2v v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = src[q];
#pragma unroll
        for (int q = 0; q < 8; ++q) acc += v[q][0] + v[q][1];
    }
    out[(size_t)w * 64 + l] = acc;
}
// the same bytes, lane l reading consecutive 16-byte chunks of each 4-kite interval block
__global__ __launch_bounds__(64) void k_coal(const double* __restrict__ a, double* __restrict__ out, int nwaves) {
    const int w = blockIdx.x, l = threadIdx.x;
    if (w >= nwaves) return;
    double acc = 0.0;
    for (int k = 0; k < 20; ++k) {
        for (int g = 0; g < 4; ++g) {
            const double2v* src = reinterpret_cast<const double2v*>(a + (((size_t)(4 * w + g) * 20 + k) * 13) * 16);
            double2v v0 = src[l];
            double2v v1 = l < 40 ? src[64 + l] : double2v{0.0, 0.0};
            acc += v0[0] + v0[1] + v1[0] + v1[1];
        }
    }
    out[(size_t)w * 64 + l] = acc;
}

int main() {
    const int kites = 4096, nwaves = kites / 4;
    const size_t nd = (size_t)kites * 20 * 13 * 16;
    double *a, *out;
    hipMalloc(&a, nd * 8); hipMalloc(&out, (size_t)nwaves * 64 * 8 * 2);
    hipMemset(a, 0, nd * 8);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto run = [&](const char* name, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        hipDeviceSynchronize();
        hipEventRecord(e0);
        const int R = 20;
        for (int i = 0; i < R; ++i) launch();
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        const double us = ms * 1e3 / R;
        printf("%-34s %8.2f us  %6.2f TB/s\n", name, us, nd * 8 / (us * 1e-6) / 1e12);
    };
    run("rows (1 wave/SIMD grid)", [&] { hipLaunchKernelGGL(k_rows, dim3(nwaves), dim3(64), 0, 0, a, out, nwaves); });
    run("coalesced (1 wave/SIMD grid)", [&] { hipLaunchKernelGGL(k_coal, dim3(nwaves), dim3(64), 0, 0, a, out, nwaves); });
    hipFree(a); hipFree(out);
    return 0;
}
