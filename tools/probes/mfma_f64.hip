// Latency / throughput probe of the fp64 building blocks of the Riccati QP on
// gfx950: v_mfma_f64_16x16x4_f64 (dependent chain, independent chains, 1..4
// waves per SIMD), dependent v_fma_f64, an LDS write->read round trip and a
// ds_bpermute of a double.  Prints cycles per operation (s_memtime ticks).
//   hipcc -O3 --offload-arch=gfx950 -o tools/bin/mfma_f64 tools/probes/mfma_f64.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int REPS = 256;

__global__ void k_mfma_dep(double* out, long long* cyc) {
    const int l = threadIdx.x;
    double a = 1.0 + 1e-9 * l, b = 1.0 - 1e-9 * l;
    d4 acc = {0, 0, 0, 0};
    long long t0 = clock64();
#pragma unroll 8
    for (int i = 0; i < REPS; ++i) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    double s = acc[0] + acc[1] + acc[2] + acc[3];
    long long t1 = clock64();
    out[blockIdx.x * blockDim.x + l] = s;
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_mfma_ind4(double* out, long long* cyc) {
    const int l = threadIdx.x;
    double a = 1.0 + 1e-9 * l, b = 1.0 - 1e-9 * l;
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    long long t0 = clock64();
#pragma unroll 4
    for (int i = 0; i < REPS / 4; ++i) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
    d4 acc = c0 + c1 + c2 + c3;
    double s = acc[0] + acc[1] + acc[2] + acc[3];
    long long t1 = clock64();
    out[blockIdx.x * blockDim.x + l] = s;
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

// dependent chain whose B operand is the previous result (true data dependence
// through the output registers, as in P -> P*A -> A^T*(P*A))
__global__ void k_mfma_dep_src(double* out, long long* cyc) {
    const int l = threadIdx.x;
    double a = 1e-3 * l;
    d4 acc = {1e-3, 0, 0, 0};
    long long t0 = clock64();
#pragma unroll 8
    for (int i = 0; i < REPS; ++i) {
        d4 z = {0, 0, 0, 0};
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, acc[0], z, 0, 0, 0);
    }
    double s = acc[0] + acc[1] + acc[2] + acc[3];
    long long t1 = clock64();
    out[blockIdx.x * blockDim.x + l] = s;
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_fma_dep(double* out, long long* cyc) {
    const int l = threadIdx.x;
    double x = 1.0 + 1e-9 * l, y = 0.999999;
    long long t0 = clock64();
#pragma unroll 16
    for (int i = 0; i < REPS; ++i) x = __builtin_fma(x, y, 1e-7);
    long long t1 = clock64();
    out[blockIdx.x * blockDim.x + l] = x;
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_fma_ind8(double* out, long long* cyc) {
    const int l = threadIdx.x;
    double x[8];
    for (int j = 0; j < 8; ++j) x[j] = 1.0 + 1e-9 * (l + j);
    const double y = 0.999999;
    long long t0 = clock64();
#pragma unroll 4
    for (int i = 0; i < REPS / 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = __builtin_fma(x[j], y, 1e-7);
    long long t1 = clock64();
    double s = 0;
    for (int j = 0; j < 8; ++j) s += x[j];
    out[blockIdx.x * blockDim.x + l] = s;
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

// LDS round trip: lane l writes, lane (l ^ 17) reads, dependent REPS times
__global__ void k_lds_rt(double* out, long long* cyc) {
    __shared__ double sm[64];
    const int l = threadIdx.x;
    double x = 1.0 + l;
    long long t0 = clock64();
    for (int i = 0; i < REPS / 8; ++i) {
        sm[l] = x;
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
        __builtin_amdgcn_wave_barrier();
        x = sm[l ^ 17] + 1.0;
        __builtin_amdgcn_wave_barrier();
    }
    long long t1 = clock64();
    out[blockIdx.x * blockDim.x + l] = x;
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_bperm(double* out, long long* cyc) {
    const int l = threadIdx.x;
    double x = 1.0 + l;
    long long t0 = clock64();
    for (int i = 0; i < REPS / 8; ++i) {
        int lo = __builtin_amdgcn_ds_bpermute(((l ^ 17) << 2), __double2loint(x));
        int hi = __builtin_amdgcn_ds_bpermute(((l ^ 17) << 2), __double2hiint(x));
        x = __hiloint2double(hi, lo) + 1.0;
    }
    long long t1 = clock64();
    out[blockIdx.x * blockDim.x + l] = x;
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

typedef void (*KFn)(double*, long long*);

static void run(const char* name, KFn k, int per_op_div, int waves_per_simd) {
    const int nblk = 256 * 4 * waves_per_simd;
    double* d; long long* c;
    hipMalloc(&d, nblk * 64 * sizeof(double));
    hipMalloc(&c, nblk * sizeof(long long));
    hipLaunchKernelGGL(k, dim3(nblk), dim3(64), 0, 0, d, c);   // warm
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(nblk), dim3(64), 0, 0, d, c);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    long long* h = new long long[nblk];
    hipMemcpy(h, c, nblk * sizeof(long long), hipMemcpyDeviceToHost);
    double mean = 0; for (int i = 0; i < nblk; ++i) mean += h[i]; mean /= nblk;
    printf("%-34s waves/SIMD %d : %8.1f cycles per op (wave view), kernel %.3f ms\n", name, waves_per_simd,
           mean / per_op_div, ms);
    delete[] h; hipFree(d); hipFree(c);
}

int main() {
    for (int w = 1; w <= 4; w *= 2) {
        run("mfma_f64 16x16x4 dependent acc", k_mfma_dep, REPS, w);
        run("mfma_f64 4 independent accs", k_mfma_ind4, REPS, w);
        run("mfma_f64 dependent via B operand", k_mfma_dep_src, REPS, w);
        run("v_fma_f64 dependent", k_fma_dep, REPS, w);
        run("v_fma_f64 8 independent", k_fma_ind8, REPS, w);
        run("lds write->read round trip", k_lds_rt, REPS / 8, w);
        run("ds_bpermute f64 (2 dwords)", k_bperm, REPS / 8, w);
    }
    return 0;
}
