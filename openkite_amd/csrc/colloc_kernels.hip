// colloc_kernels.hip -- the reference's own NLP formulation (Chebyshev-Gauss-
// Lobatto collocation, src/kite_math/pseudospectral/chebyshev.hpp:241-333 with
// the NMPF cost of kiteNMPF.cpp:100-143) evaluated for a batch of points on
// gfx950: residual G, cost J and the per-node Jacobian blocks
// of the scaled augmented ODE.
//
// One block per point, 16 lanes per collocation node: lane d pushes the dual
// direction d (13 kite states, 3 kite controls) through the RHS, so the node's
// 15 x 19 block of d SODE / d [x, u] comes out of one pass; the residual rows
// and the quadrature of the Lagrange term use the primal part every lane
// carries.  CompDiff (nodes x nodes) and the node weights of the quadrature
// come from the host in a small device table.
#include <hip/hip_runtime.h>
#include <math.h>

#include "kite_model.hpp"
#include "rti_kernels.hpp"

namespace kite {

constexpr int CL_MAXN = 32;         // nodes per point (blockDim = 16 * nodes)

__device__ __forceinline__ void colloc_path(const CollocConst& C, double th, double P[3]) {
    double s, c;
    sincos(th, &s, &c);
    const double qw = C.pq[0];
    const V3<double> qu{C.pq[1], C.pq[2], C.pq[3]};
    const double ww_uu = qw * qw - dot3(qu, qu);
    double pc[3], dpc[3];
    path_curve(C.path_K, C.path_R, C.path_alt, C.pF, c, s, pc, dpc);
    const V3<double> p = rot_body(qw, qu, ww_uu, V3<double>{pc[0], pc[1], pc[2]});
    P[0] = p.x; P[1] = p.y; P[2] = p.z;
}

__global__ __launch_bounds__(16 * CL_MAXN) void k_colloc(ModelConst P, CollocConst C, int count,
                                                         const double* __restrict__ tab,   // CD (n x n) | wn (n)
                                                         const double* __restrict__ z, double* __restrict__ G,
                                                         double* __restrict__ J, double* __restrict__ jac) {
    __shared__ double sJ[CL_MAXN];
    const int pt = blockIdx.x;
    const int i = threadIdx.x >> 4, d = threadIdx.x & 15;
    const int n = C.nodes;
    const int nz = n * 19;
    const double* zp = z + (size_t)pt * nz;
    const double* X = zp;                  // n x 15 (formulation variables)
    const double* U = zp + n * 15;         // n x 4
    const double* xs = X + i * 15;
    const double* us = U + i * 4;

    // physical point and dual direction d
    Dual xx[NK], uu[NKU], ff[NK];
    for (int c = 0; c < NK; ++c) xx[c] = mk(xs[c] * C.iSx[c], d == c ? C.iSx[c] : 0.0);
    for (int c = 0; c < NKU; ++c) uu[c] = mk(us[c] * C.iSu[c], d == NK + c ? C.iSu[c] : 0.0);
    kite_rhs<Dual>(P, xx, uu, ff);

    // scaled augmented ODE value (every lane has it)
    double sode[15];
    for (int r = 0; r < NK; ++r) sode[r] = C.Sx[r] * ff[r].v;
    sode[13] = C.Sx[13] * (xs[14] * C.iSx[14]);        // theta'    = thetadot
    sode[14] = C.Sx[14] * (us[3] * C.iSu[3]);          // thetadot' = Uv

    // residual rows G_i = sum_j CD[i][j] X_j - t_scale SODE_i (lanes 0..14)
    if (d < 15) {
        double t = 0.0;
        for (int j = 0; j < n; ++j) t = fma(tab[i * n + j], X[j * 15 + d], t);
        G[(size_t)pt * n * 15 + i * 15 + d] = t - C.t_scale * sode[d];
    }
    // Jacobian block d SODE_i / d [x, u] (15 x 19)
    if (jac) {
        double* jb = jac + ((size_t)pt * n + i) * 15 * 19;
        const int colj = d < NK ? d : 15 + (d - NK);
        for (int r = 0; r < NK; ++r) jb[r * 19 + colj] = C.Sx[r] * ff[r].t;
        if (d == 0) {
            for (int r = 0; r < NK; ++r) { jb[r * 19 + 13] = 0.0; jb[r * 19 + 14] = 0.0; jb[r * 19 + 18] = 0.0; }
            for (int c = 0; c < 19; ++c) { jb[13 * 19 + c] = 0.0; jb[14 * 19 + c] = 0.0; }
            jb[13 * 19 + 14] = C.Sx[13] * C.iSx[14];
            jb[14 * 19 + 18] = C.Sx[14] * C.iSu[3];
        }
    }
    // cost: node weight x Lagrange (+ Mayer at node 0), chebyshev.hpp:280-333
    if (d == 0) {
        double Pp[3];
        colloc_path(C, xs[13] * C.iSx[13], Pp);
        double q = 0.0;
        for (int a = 0; a < 3; ++a) {
            const double res = C.Sx[6 + a] * Pp[a] - xs[6 + a];
            q += C.Q[a] * res * res;
        }
        double L = q + C.W * (C.vref - xs[14]) * (C.vref - xs[14]);
        if (C.use_R)
            for (int c = 0; c < 4; ++c) L += C.R[c] * us[c] * us[c];
        double v = tab[n * n + i] * L;
        if (i == 0) v += C.mayer_scale * q;
        sJ[i] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int k = 0; k < n; ++k) t += sJ[k];
        J[pt] = t;
    }
}

hipError_t launch_colloc(const ModelConst& P, const CollocConst& C, int count, const double* tab, const double* z,
                         double* G, double* J, double* jac, hipStream_t s) {
    if (C.nodes < 1 || C.nodes > CL_MAXN) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_colloc, dim3(count), dim3(16 * C.nodes), 0, s, P, C, count, tab, z, G, J, jac);
    return hipGetLastError();
}

}  // namespace kite
