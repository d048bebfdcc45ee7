// ekf_kernels.hip -- batched extended Kalman filter of the kite
// on gfx950: KiteEKF::propagate + KiteEKF::_estimate
// (src/kite_estimation/kiteEKF.cpp:75-126) for `count` kites in one launch.
//
//   propagate  x+ = RK4(x, u, dt) (one step, kite.cpp:332-338),
//              A  = I + J(x) dt,  P+ = A P A' + W
//   update     y = z - H x+,  S = H P+ H' + V,  K = P+ H' S^-1,
//              x = x+ + K y,  P = (I - K H) P+      with H = [0_{7x6} I_7]
//
// Lane layout: one lane per (kite, column j of the 13 x 13 matrices); 16 lanes
// per kite (13 used), 4 kites per wavefront.  Lane j computes column j of the
// Jacobian with one dual-number pass of the RHS, then column j of A P and of
// A P A' from the matrices shared through LDS (13 x 14 per kite, LDS
// broadcast reads); the 7 x 7 innovation covariance is factored per lane in
// registers.  HBM per kite: x, u, z, P in and x, P out = 2 x 1.4 KB.
#include <hip/hip_runtime.h>
#include <math.h>

#include "kite_model.hpp"
#include "rti_kernels.hpp"

namespace kite {

constexpr int EKF_T = 64;           // threads per block = 4 kites x 16 lanes
constexpr int EKF_LD = 14;          // LDS row stride of a 13 x 13 matrix

__global__ __launch_bounds__(EKF_T, 2) void k_ekf(ModelConst P, int count, double dt, double* __restrict__ x,
                                                   const double* __restrict__ u, double* __restrict__ Pc,
                                                   const double* __restrict__ z, const double* __restrict__ W,
                                                   const double* __restrict__ V) {
    __shared__ double sA[4][NK * EKF_LD];
    __shared__ double sN[4][NK * EKF_LD];
    const int kk = threadIdx.x >> 4, j = threadIdx.x & 15;
    const int b = blockIdx.x * 4 + kk;
    const bool kite = b < count;
    const bool col = kite && j < NK;
    double* sa = sA[kk];
    double* sn = sN[kk];

    double xv[NK], uv[NKU];
    for (int i = 0; i < NK; ++i) xv[i] = kite ? x[(size_t)b * NK + i] : 0.0;
    for (int i = 0; i < NKU; ++i) uv[i] = kite ? u[(size_t)b * NKU + i] : 0.0;

    // column j of A = I + J dt at the estimate (kiteEKF.cpp:93)
    if (col) {
        Dual xx[NK], uu[NKU], ff[NK];
        for (int i = 0; i < NK; ++i) xx[i] = mk(xv[i], i == j ? 1.0 : 0.0);
        for (int i = 0; i < NKU; ++i) uu[i] = mk(uv[i], 0.0);
        kite_rhs<Dual>(P, xx, uu, ff);
        for (int i = 0; i < NK; ++i) sa[i * EKF_LD + j] = ff[i].t * dt + (i == j ? 1.0 : 0.0);
    }
    // x+ = one RK4 step over dt (kitemath.cpp:36-51), every lane of the kite
    double xn[NK];
    {
        double k[NK], xs[NK];
        for (int i = 0; i < NK; ++i) { xn[i] = xv[i]; xs[i] = xv[i]; }
#pragma unroll 1
        for (int st = 0; st < 4; ++st) {
            kite_rhs<double>(P, xs, uv, k);
            const double wa = (st == 0 || st == 3) ? dt / 6.0 : dt / 3.0;
            const double wn = (st < 2) ? 0.5 * dt : dt;
            for (int i = 0; i < NK; ++i) { xn[i] += wa * k[i]; xs[i] = xv[i] + wn * k[i]; }
        }
    }
    double pcol[NK];
    for (int i = 0; i < NK; ++i) pcol[i] = col ? Pc[((size_t)b * NK + i) * NK + j] : 0.0;
    __syncthreads();
    // (A P)[:, j]
    if (col) {
        for (int i = 0; i < NK; ++i) {
            double t = 0.0;
            for (int k = 0; k < NK; ++k) t = fma(sa[i * EKF_LD + k], pcol[k], t);
            sn[i * EKF_LD + j] = t;
        }
    }
    __syncthreads();
    // P+[:, j] = sum_k (A P)[:, k] A[j][k] + W[:, j]
    if (col) {
        for (int i = 0; i < NK; ++i) {
            double t = W[i * NK + j];
            for (int k = 0; k < NK; ++k) t = fma(sn[i * EKF_LD + k], sa[j * EKF_LD + k], t);
            pcol[i] = t;
        }
    }
    if (z) {
        __syncthreads();
        if (col) for (int i = 0; i < NK; ++i) sn[i * EKF_LD + j] = pcol[i];
        __syncthreads();
        // S = P+[6:13, 6:13] + V, Cholesky in registers (lower, row-major packed)
        double L[7][7];
        for (int a = 0; a < 7; ++a)
            for (int c = 0; c <= a; ++c) L[a][c] = kite ? sn[(6 + a) * EKF_LD + 6 + c] + V[a * 7 + c] : (a == c);
        for (int c = 0; c < 7; ++c) {
            double d = L[c][c];
            for (int k = 0; k < c; ++k) d -= L[c][k] * L[c][k];
            d = sqrt(d);
            L[c][c] = d;
            for (int a = c + 1; a < 7; ++a) {
                double t = L[a][c];
                for (int k = 0; k < c; ++k) t -= L[a][k] * L[c][k];
                L[a][c] = t / d;
            }
        }
        auto solve = [&](double r[7]) {          // r <- S^-1 r
            for (int a = 0; a < 7; ++a) {
                double t = r[a];
                for (int k = 0; k < a; ++k) t -= L[a][k] * r[k];
                r[a] = t / L[a][a];
            }
            for (int a = 6; a >= 0; --a) {
                double t = r[a];
                for (int k = a + 1; k < 7; ++k) t -= L[k][a] * r[k];
                r[a] = t / L[a][a];
            }
        };
        // P[:, j] = P+[:, j] - P+[:, 6:13] S^-1 P+[6:13, j]
        if (col) {
            double c7[7];
            for (int a = 0; a < 7; ++a) c7[a] = pcol[6 + a];
            solve(c7);
            for (int i = 0; i < NK; ++i) {
                double t = pcol[i];
                for (int a = 0; a < 7; ++a) t = fma(-sn[i * EKF_LD + 6 + a], c7[a], t);
                pcol[i] = t;
            }
        }
        // x = x+ + P+[:, 6:13] S^-1 (z - x+[6:13])
        if (kite && j == 0) {
            double y[7];
            for (int a = 0; a < 7; ++a) y[a] = z[(size_t)b * 7 + a] - xn[6 + a];
            solve(y);
            for (int i = 0; i < NK; ++i) {
                double t = xn[i];
                for (int a = 0; a < 7; ++a) t = fma(sn[i * EKF_LD + 6 + a], y[a], t);
                xn[i] = t;
            }
        }
    }
    if (col)
        for (int i = 0; i < NK; ++i) Pc[((size_t)b * NK + i) * NK + j] = pcol[i];
    if (kite && j == 0)
        for (int i = 0; i < NK; ++i) x[(size_t)b * NK + i] = xn[i];
}

hipError_t launch_ekf(const ModelConst& P, int count, double dt, double* x, const double* u, double* Pc,
                      const double* z, const double* W, const double* V, hipStream_t s) {
    hipLaunchKernelGGL(k_ekf, dim3((count + 3) / 4), dim3(EKF_T), 0, s, P, count, dt, x, u, Pc, z, W, V);
    return hipGetLastError();
}

}  // namespace kite
