// FETCH_SIZE / WRITE_SIZE calibration for the load shapes of k_qp_ric.
//
// bench.py's traffic figure doubles FETCH_SIZE (the microarchitecture guide's
// rule for 16-B/lane coalesced streaming reads).  k_qp_ric streams Z_k by
// 8-B/lane loads (512 B contiguous per wave instruction, ric_load_Z) and
// re-reads it from beyond L2 a few dozen times per launch.  This program
// reads buffers of known size in those shapes so that rocprofv3's counters
// can be converted to bytes for each shape:
//   k_read8   each byte of a 1 GiB buffer once, 8 B/lane  (HBM, > Infinity Cache)
//   k_read16  the same, 16 B/lane
//   k_reread8 a 64 MiB buffer 8 times, 8 B/lane, each pass by other CUs
//             (> one XCD's 4 MiB L2, < the 256 MiB Infinity Cache): whether
//             Infinity-Cache hits are counted
//   k_write8  1 GiB written once, 8 B/lane
// Each kernel writes one double per wave of its sum so nothing is elided.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(1); } } while (0)

constexpr int WAVES = 8192;         // 2048 workgroups x 4 waves; each wave strides the buffer

__global__ __launch_bounds__(256) void k_read8(const double* __restrict__ a, size_t n, double* __restrict__ out) {
    const size_t w = (blockIdx.x * 4 + threadIdx.x / 64), l = threadIdx.x & 63;
    double s = 0.0;
    for (size_t i = w * 64 + l; i < n; i += (size_t)WAVES * 64) s += a[i];
    if (s == 1.2345) out[w * 64 + l] = s;       // practically never; keeps the loads
}
__global__ __launch_bounds__(256) void k_read16(const double2* __restrict__ a, size_t n2, double* __restrict__ out) {
    const size_t w = (blockIdx.x * 4 + threadIdx.x / 64), l = threadIdx.x & 63;
    double s = 0.0;
    for (size_t i = w * 64 + l; i < n2; i += (size_t)WAVES * 64) { const double2 v = a[i]; s += v.x + v.y; }
    if (s == 1.2345) out[w * 64 + l] = s;
}
// pass p of wave w reads chunk (w + p * WAVES / 8) % WAVES: the 8 passes of a
// chunk come from waves of 8 different workgroup ranges (other CUs / XCDs)
__global__ __launch_bounds__(256) void k_reread8(const double* __restrict__ a, size_t n, double* __restrict__ out) {
    const size_t w = (blockIdx.x * 4 + threadIdx.x / 64), l = threadIdx.x & 63;
    const size_t chunk = n / WAVES;
    double s = 0.0;
    for (int p = 0; p < 8; ++p) {
        const size_t c = (w + (size_t)p * (WAVES / 8) + (size_t)p * 37) % WAVES;
        const double* b = a + c * chunk;
        for (size_t i = l; i < chunk; i += 64) s += b[i];
    }
    if (s == 1.2345) out[w * 64 + l] = s;
}
__global__ __launch_bounds__(256) void k_write8(double* __restrict__ a, size_t n) {
    const size_t w = (blockIdx.x * 4 + threadIdx.x / 64), l = threadIdx.x & 63;
    for (size_t i = w * 64 + l; i < n; i += (size_t)WAVES * 64) a[i] = (double)i;
}

int main() {
    const size_t big = (size_t)1 << 30, small = (size_t)64 << 20;
    double *a, *b, *out;
    CK(hipMalloc(&a, big));
    CK(hipMalloc(&b, small));
    CK(hipMalloc(&out, (size_t)WAVES * 64 * sizeof(double)));
    CK(hipMemset(a, 0, big));
    CK(hipMemset(b, 0, small));
    const dim3 grid(WAVES / 4), block(256);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto timed = [&](const char* name, double bytes, auto launch) {
        launch();                                   // warm (clock, TLB)
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("{\"kernel\": \"%s\", \"bytes_per_launch\": %.0f, \"ms\": %.4f, \"GBps\": %.1f}\n", name, bytes, ms,
                    bytes / (ms * 1e6));
    };
    timed("k_read8", (double)big, [&] { k_read8<<<grid, block>>>(a, big / 8, out); });
    timed("k_read16", (double)big, [&] { k_read16<<<grid, block>>>((const double2*)a, big / 16, out); });
    timed("k_reread8", 8.0 * (double)small, [&] { k_reread8<<<grid, block>>>(b, small / 8, out); });
    timed("k_write8", (double)big, [&] { k_write8<<<grid, block>>>(a, big / 8); });
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipFree(a)); CK(hipFree(b)); CK(hipFree(out));
    return 0;
}
