// ubench_qp.hip -- latency micro-benchmarks of the k_qp_tiled building blocks
// (tools only: one wave, dependent repetitions, shader-clock cycles per call).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -o /tmp/ubench_qp tools/ubench_qp.hip
// Compiles the product kernels TU in (for the device helpers).
#include "../openkite_amd/csrc/rti_kernels.hip"

#include <cstdio>
#include <vector>

namespace kite {

enum { UB_CHOL = 0, UB_PIVOT, UB_FWD, UB_BWD, UB_PANEL, UB_SYMV, UB_ROWSUM, UB_COUNT };

__global__ __launch_bounds__(64, 1) void k_ubench(int which, int reps, double* sink, unsigned long long* cyc) {
    __shared__ double sT[QP_NTA * 16 * TLD];
    __shared__ double sP[(QP_NTA - 1) * 16 * TLD];
    __shared__ double sV[2 * QNA];
    const int l = threadIdx.x, cl = l & 15, rg = l >> 4;
    double4v a;
#pragma unroll
    for (int r = 0; r < 4; ++r) a[r] = (rg + 4 * r == cl) ? 16.0 : 1.0 / (1.0 + abs(rg + 4 * r - cl));
    for (int i = l; i < QP_NTA * 16 * TLD; i += 64) sT[i] = 1e-3 * (i % 7);
    for (int i = l; i < (QP_NTA - 1) * 16 * TLD; i += 64) sP[i] = 1e-3 * (i % 5);
    for (int i = l; i < 2 * QNA; i += 64) sV[i] = 1.0 + 1e-3 * i;
    double4v Mt[QP_NTILE];
#pragma unroll
    for (int t = 0; t < QP_NTILE; ++t) Mt[t] = a;
    wave_sync();
    double acc = 0.0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (which == UB_CHOL) {
        for (int it = 0; it < reps; ++it) {
            double4v m = a, x;
            chol_tile(m, x, l);
            a[0] += 1e-300 * x[0];                     // carried dependency
        }
        acc = a[0];
    } else if (which == UB_PIVOT) {                      // 16 dependent rsq + 2 Newton
        double p = 2.0 + l;
        for (int it = 0; it < reps; ++it)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const double piv = piv_fix(dpp_d<0x150 + 3>(p));
                double inv = __builtin_amdgcn_rsq(piv);
                inv = inv * fma(-0.5 * piv, inv * inv, 1.5);
                inv = inv * fma(-0.5 * piv, inv * inv, 1.5);
                p = fma(p, inv, 1.0);
            }
        acc = p;
    } else if (which == UB_FWD) {
        const double* tl = sT + cl * TLD + rg;
        for (int it = 0; it < reps; ++it) {
            double y[QP_NTA];
            fwd_solve(Mt, tl, sV, sV + QNA, rg, y);
            Mt[0][0] += 1e-300 * y[QP_NTA - 1];
        }
        acc = Mt[0][0];
    } else if (which == UB_BWD) {
        const double* tl = sT + cl * TLD + rg;
        double y[QP_NTA];
#pragma unroll
        for (int K = 0; K < QP_NTA; ++K) y[K] = 1.0 + K;
        for (int it = 0; it < reps; ++it) {
            double x[QP_NTA][4];
            bwd_solve(Mt, tl, y, x);
            y[QP_NTA - 1] += 1e-300 * x[0][0];
        }
        acc = y[QP_NTA - 1];
    } else if (which == UB_PANEL) {                      // one step K = 0: stage, panels, store
        for (int it = 0; it < reps; ++it) {
#pragma unroll
            for (int I = 1; I < QP_NTA; ++I) tile_store(sP + (I - 1) * 16 * TLD, Mt[TI(I, 0)], l);
            wave_sync();
            double4v pacc[QP_NTA - 1];
#pragma unroll
            for (int I = 1; I < QP_NTA; ++I) {
                pacc[I - 1] = double4v{0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int s = 0; s < 4; ++s)
                    pacc[I - 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(tile_frag(sP + (I - 1) * 16 * TLD, s, l),
                                                                       tile_frag(sT, s, l), pacc[I - 1], 0, 0, 0);
            }
            wave_sync();
#pragma unroll
            for (int I = 1; I < QP_NTA; ++I) {
                Mt[TI(I, 0)] = pacc[I - 1];
                tile_store(sP + (I - 1) * 16 * TLD, pacc[I - 1], l);
            }
            wave_sync();
        }
        acc = Mt[TI(4, 0)][0];
    } else if (which == UB_SYMV) {
        for (int it = 0; it < reps; ++it) {
            tile_symv(Mt, sV, sV + QNA, l);
            Mt[0][0] += 1e-300 * sV[QNA + 5];
        }
        acc = Mt[0][0];
    } else if (which == UB_ROWSUM) {                     // 16 dependent row_sum16 + col_sum4
        double v = 1.0 + l;
        for (int it = 0; it < reps; ++it)
#pragma unroll
            for (int q = 0; q < 16; ++q) v = col_sum4(row_sum16(v)) * 1e-3;
        acc = v;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    sink[l] = acc;
    if (l == 0) cyc[0] = t1 - t0;
}

}  // namespace kite

int main() {
    const char* names[] = {"chol_tile (16x16, incl. T = L^-1)", "16 pivots rsq+2 Newton (chain)",
                           "fwd_solve (5 tiles)", "bwd_solve (5 tiles)", "panel step K=0 (stage+4 panels+store)",
                           "tile_symv (15 tiles)", "16 x (row_sum16 + col_sum4)"};
    double* sink;
    unsigned long long* cyc;
    (void)hipMalloc(&sink, 64 * sizeof(double));
    (void)hipMalloc(&cyc, sizeof(unsigned long long));
    const int reps = 200;
    for (int w = 0; w < kite::UB_COUNT; ++w) {
        unsigned long long c = 0;
        for (int rep = 0; rep < 3; ++rep) {          // last of 3 (warm)
            hipLaunchKernelGGL(kite::k_ubench, dim3(1), dim3(64), 0, 0, w, reps, sink, cyc);
            (void)hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
        }
        printf("%-40s %10.0f cycles per call\n", names[w], (double)c / reps);
    }
    return 0;
}
