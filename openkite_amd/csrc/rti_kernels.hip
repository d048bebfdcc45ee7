// rti_kernels.hip -- batched RTI step for the openKITE kite NMPC on gfx950.
//
// One RTI step = k_prologue -> k_rk4_sens2 -> k_condense -> k_qp (see
// DESIGN.md).  Replaces KiteNMPF::computeControl's NLP_Solver(ARG) call
// (src/kite_control/kiteNMPF.cpp:199-316).
//
// Memory layout (HBM, fp64): every per-instance object is contiguous and the
// instances are stacked (instance-major), i.e. exactly the host API layout:
//   X   [B][N+1][15]   linearisation / solution trajectory (physical units)
//   U   [B][N][4]
//   AB  [B][N][13][16] d x+_kite / d [x_kite(13) | u_kite(3)]  per interval
//   DEF [B][N][13]     multiple-shooting defects  x+(x_k,u_k) - x_{k+1}
//   Hs  [B][n][n], hs [B][n], Cr [B][N][n], cl/cu [B][N]  condensed QP
// with n = 4N+2 decision variables in GPU column order
//   [T,dE,dR]_k (3N) | Uv_k (N) | theta_0 | thetadot_0.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <type_traits>

#include "kite_model.hpp"
#include "rti_kernels.hpp"
#include "rti_device.hpp"

namespace kite {

// findClosestPointOnPath (kiteNMPF.cpp:358-391): <= 10 gradient steps of 1/4 on
// 1/2 ||P(theta) - r|| (the non-squared norm as written, kiteNMPF.cpp:361)
__device__ double closest_point_dev(const RtiConst& C, double px, double py, double pz, double guess) {
    auto grad = [&](double th) {
        double P[3], dP[3];
        path_eval(C, th, P, dP);
        const double e0 = P[0] - px, e1 = P[1] - py, e2 = P[2] - pz;
        const double nrm = sqrt(e0 * e0 + e1 * e1 + e2 * e2);
        return 0.5 * (e0 * dP[0] + e1 * dP[1] + e2 * dP[2]) / nrm;
    };
    double th = guess;
    double g = grad(th);
    if (fabs(g) < 1e-2) { th = M_PI_2 + 0.1; g = grad(th); }
    int counter = 0;
    while (fabs(g) >= 1e-2) {
        ++counter;
        th -= 0.25 * g;
        g = grad(th);
        if (counter > 10) break;
    }
    return th;
}

// primal RK4 of the augmented 15-state model, M substeps of length h (WIND:
// the constant world-frame wind wnd[0..2] of this kite, kite_model.hpp)
template <bool WIND = false>
__device__ void rk4_primal(const ModelConst& P, const double* x0, const double* u, double h, int M,
                           double* xo, const double* wnd = nullptr) {
    double x[NX], xs[NX], acc[NX], k[NK];
#pragma unroll
    for (int i = 0; i < NX; ++i) x[i] = x0[i];
    for (int m = 0; m < M; ++m) {
#pragma unroll
        for (int i = 0; i < NX; ++i) { xs[i] = x[i]; acc[i] = x[i]; }
#pragma unroll 1
        for (int st = 0; st < 4; ++st) {
            kite_rhs<double, WIND>(P, xs, u, k, wnd);
            const double kt = xs[14], kth = u[3];   // theta' = thetadot, thetadot' = Uv
            const double wa = (st == 0 || st == 3) ? h / 6.0 : h / 3.0;
            const double wn = (st < 2) ? 0.5 * h : h;
#pragma unroll
            for (int i = 0; i < NK; ++i) { acc[i] += wa * k[i]; xs[i] = x[i] + wn * k[i]; }
            acc[13] += wa * kt; acc[14] += wa * kth;
            xs[13] = x[13] + wn * kt; xs[14] = x[14] + wn * kth;
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) x[i] = acc[i];
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) xo[i] = x[i];
}

// ---------------------------------------------------------------------------
// k_prologue: one wavefront per instance.  theta wrap (kiteNMPF.cpp:209-221),
// min speed clamp (nmpf_node.cpp:241-243), warm-start shift or cold start
// (controls at the bound midpoint kiteNMPF.cpp:192-196, states by forward
// simulation), x_0 pinned, theta/thetadot re-simulated exactly.  The per-kite
// scalar logic runs on lane 0; the warm-start shift (the bulk of the bytes)
// is a coalesced copy by the whole wave.
//
// FULL = false is the warm step without delay compensation, the common case:
// no forward simulation is compiled in, so the kernel holds few registers and
// runs at full occupancy (the full variant's inlined RK4 and closest-point
// search take ~300 VGPRs, one wave per SIMD).  A kite it finds flagged for a
// cold restart (status bit 1) goes on the cold list (cold[0] = count, entries
// from cold[1]) instead, and k_prologue_cold runs the full variant for those.
// Both variants execute the same arithmetic for a kite they both handle.
// ---------------------------------------------------------------------------
template <bool FULL>
__device__ __forceinline__ void prologue_kite(const ModelConst& P, const RtiConst& C, int b, int warm,
                                              const double* __restrict__ x0in, double* __restrict__ X,
                                              double* __restrict__ U, int32_t* __restrict__ status,
                                              const double* __restrict__ wind, int32_t* __restrict__ cold,
                                              double* sx0, double* sUv, int* sWarm_, int B = 0) {
    int& sWarm = *sWarm_;
    const int l = threadIdx.x;
    const int N = C.N;
    double* Xb = X + (size_t)b * (N + 1) * NX;
    double* Ub = U + (size_t)b * N * NU;
    int32_t st = 0;
    if constexpr (!FULL) {
        // launched on warm steps only: a kite flagged for a cold restart leaves
        // for the cold list (block-uniform, the whole wave returns)
        if (l == 0) sWarm = (status[b] & 1) ? -1 : 1;
        __syncthreads();
        if (sWarm < 0) {
            if (l == 0) {
                const int slot = atomicAdd(cold, 1);   // < B: launch_prologue zeroes the count first
                if (slot < B) cold[1 + slot] = b;
            }
            return;
        }
        __syncthreads();
    }
    if (l == 0) {
        double x0[NX];
        for (int i = 0; i < NX; ++i) x0[i] = x0in[(size_t)b * NX + i];
        int wm = warm;
        if (FULL && wm && (status[b] & 1)) {
            // a non-finite plan (a NaN iterate of a previous step) cannot seed a
            // warm start: restart this kite cold, theta re-initialised by the
            // closest point and thetadot = 0 (the node's init, nmpf_node.cpp:225-236).
            // The previous epilogue flagged it (KITE_ST_NAN: non-finite X or U);
            // kite_nmpc_set_solution flags injected plans the same way.
            wm = 0;
            st |= 64;
            x0[13] = closest_point_dev(C, x0[6], x0[7], x0[8], isfinite(x0[13]) ? x0[13] : 0.0);
            x0[14] = 0.0;
        }
        if (FULL && wm && C.delay > 0.0) {
            // transport-delay compensation (nmpf_node.cpp:206-221): predict the
            // measured kite state over `delay` under the previous u(t0); theta,
            // thetadot from the previous trajectory at t0 + delay
            const double up[NU] = {Ub[0], Ub[1], Ub[2], 0.0};
            double xp[NX];
            if (wind) rk4_primal<true>(P, x0, up, C.delay / C.delay_steps, C.delay_steps, xp, wind + 3 * b);
            else rk4_primal(P, x0, up, C.delay / C.delay_steps, C.delay_steps, xp);
            for (int i = 0; i < 13; ++i) x0[i] = xp[i];
            x0[13] = Xb[C.delay_node * NX + 13];
            x0[14] = Xb[C.delay_node * NX + 14];
        }
        const double twopi = 2.0 * M_PI;
        if (x0[13] > twopi) { x0[13] -= twopi; st |= 16; }
        else if (x0[13] < -twopi) { x0[13] += twopi; st |= 16; }
        if (x0[0] < C.min_speed) { x0[0] = C.min_speed; st |= 4; }
        if (FULL && !wm) {
            for (int k = 0; k < N; ++k)
                for (int j = 0; j < NU; ++j) Ub[k * NU + j] = 0.5 * (C.lbu[j] + C.ubu[j]);
            for (int i = 0; i < NX; ++i) Xb[i] = x0[i];
            for (int k = 0; k < N; ++k) {
                if (wind) rk4_primal<true>(P, &Xb[k * NX], &Ub[k * NU], C.h, C.M, &Xb[(k + 1) * NX], wind + 3 * b);
                else rk4_primal(P, &Xb[k * NX], &Ub[k * NU], C.h, C.M, &Xb[(k + 1) * NX]);
            }
            for (int k = 0; k < N; ++k) sUv[k] = Ub[k * NU + 3];
        } else if (!C.shift) {
            for (int k = 0; k < N; ++k) sUv[k] = Ub[k * NU + 3];
        }
        for (int i = 0; i < NX; ++i) sx0[i] = x0[i];
        sWarm = wm;
    }
    __syncthreads();
    const bool wm = sWarm != 0;
    if (wm && C.shift) {
        // in-place shift by one node / one interval, the last duplicated: all
        // loads of the wave complete before any store (the barrier's fence
        // orders them for the compiler and the memory pipeline; lane l stores
        // elements other lanes loaded)
        constexpr int XS = (KITE_NMAX * NX + 63) / 64, US = (KITE_NMAX * NU + 63) / 64;
        double xv[XS], uv[US];
#pragma unroll
        for (int q = 0; q < XS; ++q) {
            const int e = l + 64 * q;
            xv[q] = e < N * NX ? Xb[NX + e] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < US; ++q) {
            const int e = l + 64 * q;
            uv[q] = e < (N - 1) * NU ? Ub[NU + e] : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < XS; ++q) {
            const int e = l + 64 * q;
            if (e < N * NX) Xb[e] = xv[q];
        }
#pragma unroll
        for (int q = 0; q < US; ++q) {
            const int e = l + 64 * q;
            if (e < (N - 1) * NU) {
                Ub[e] = uv[q];
                if (e % NU == 3) sUv[e / NU] = uv[q];
            }
        }
        if (l == 0) sUv[N - 1] = Ub[(N - 1) * NU + 3];      // the last interval keeps its control
    }
    __syncthreads();
    if (l < NX) Xb[l] = sx0[l];
    if (l == 0) {
        double th = sx0[13], thd = sx0[14];
        for (int k = 0; k < N; ++k) {
            const double uv = sUv[k];
            const double thn = th + C.dt * thd + 0.5 * C.dt * C.dt * uv;
            const double thdn = thd + C.dt * uv;
            Xb[(k + 1) * NX + 13] = thn;
            Xb[(k + 1) * NX + 14] = thdn;
            th = thn; thd = thdn;
        }
        status[b] = st;
    }
}

__global__ __launch_bounds__(64) void k_prologue(ModelConst P, RtiConst C, int B, int warm,
                                                 const double* __restrict__ x0in,
                                                 double* __restrict__ X, double* __restrict__ U,
                                                 int32_t* __restrict__ status, const double* __restrict__ wind) {
    __shared__ double sx0[NX];
    __shared__ double sUv[KITE_NMAX];
    __shared__ int sWarm;
    if ((int)blockIdx.x >= B) return;
    prologue_kite<true>(P, C, blockIdx.x, warm, x0in, X, U, status, wind, nullptr, sx0, sUv, &sWarm);
}
// warm step, no delay compensation (run_step's common case)
__global__ __launch_bounds__(64) void k_prologue_warm(ModelConst P, RtiConst C, int B,
                                                      const double* __restrict__ x0in,
                                                      double* __restrict__ X, double* __restrict__ U,
                                                      int32_t* __restrict__ status, int32_t* __restrict__ cold) {
    __shared__ double sx0[NX];
    __shared__ double sUv[KITE_NMAX];
    __shared__ int sWarm;
    if ((int)blockIdx.x >= B) return;
    prologue_kite<false>(P, C, blockIdx.x, 1, x0in, X, U, status, nullptr, cold, sx0, sUv, &sWarm, B);
}
// the kites k_prologue_warm put on the cold list, one per block in a
// grid-stride loop (normally none: every block reads cold[0] = 0 and leaves)
__global__ __launch_bounds__(64) void k_prologue_cold(ModelConst P, RtiConst C, const double* __restrict__ x0in,
                                                      double* __restrict__ X, double* __restrict__ U,
                                                      int32_t* __restrict__ status,
                                                      const double* __restrict__ wind,
                                                      const int32_t* __restrict__ cold, int B) {
    __shared__ double sx0[NX];
    __shared__ double sUv[KITE_NMAX];
    __shared__ int sWarm;
    const int n = min(cold[0], B);
    for (int i = blockIdx.x; i < n; i += gridDim.x) {
        prologue_kite<true>(P, C, cold[1 + i], 1, x0in, X, U, status, wind, nullptr, sx0, sUv, &sWarm);
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// k_rk4_sens2: the sensitivity kernel.  RK4 (kitemath.cpp:36-51) with M
// substeps of the 13-state kite ODE under constant u_k, carried with forward
// tangents in the 16 directions [x_kite (13) | u_kite (3)] -> [A_k | B_k] and
// the defect x+ - x_{k+1}; theta/thetadot/Uv (an exact double integrator) are
// handled analytically in k_condense.
// ---------------------------------------------------------------------------
// fp64 sensitivities, two tangent directions per lane (Dual2): 8 lanes per
// (instance, interval) carry directions (2d, 2d+1) of [x_kite (13) | u_kite
// (3)], so the primal RHS and its transcendentals run once per two tangents
// (the 16-lane form recomputed them 16 times).  At 1 wave per SIMD the RK4
// state (value, 2 tangents, 2 accumulator tangents) stays in registers: no
// LDS.  Lane d writes columns 2d, 2d+1 of [A_k | B_k]; lane 0 the defect.
constexpr int RK2_T = 64;                 // threads per block = 8 instances x 8 direction pairs
// DT: Dual2 (fp64) or DualF2 (fp32 sensitivities, config sens_fp32 = 1; the
// defects then come from k_defects in fp64), ST its scalar
// WIND: per-kite world-frame wind wind[3 b .. 3 b + 2] (wind-field sweeps)
template <class DT, class ST, bool WIND = false>
__global__ __launch_bounds__(RK2_T, 1) void k_rk4_sens2(ModelConst P, int B, int N, int M, double h,
                                                        const double* __restrict__ X,
                                                        const double* __restrict__ U,
                                                        double* __restrict__ AB, double* __restrict__ DEF,
                                                        const double* __restrict__ wind = nullptr) {
    const int d = threadIdx.x & 7;
    const int b = blockIdx.x * (RK2_T / 8) + (threadIdx.x >> 3);
    const int k = blockIdx.y;
    if (b >= B) return;
    const double* xk = X + ((size_t)b * (N + 1) + k) * NX;
    const double* uk = U + ((size_t)b * N + k) * NU;
    const int d0 = 2 * d, d1 = 2 * d + 1;
    const ST one = ST(1), zero = ST(0), hs = ST(h);
    DT x[NK], u[NKU];
#pragma unroll
    for (int i = 0; i < NK; ++i) x[i] = DT(ST(xk[i]), d0 == i ? one : zero, d1 == i ? one : zero);
#pragma unroll
    for (int j = 0; j < NKU; ++j) u[j] = DT(ST(uk[j]), d0 == NK + j ? one : zero, d1 == NK + j ? one : zero);
#pragma unroll 1
    for (int m = 0; m < M; ++m) {
        DT xs[NK], acc[NK], kv[NK];
#pragma unroll
        for (int i = 0; i < NK; ++i) { xs[i] = x[i]; acc[i] = x[i]; }
#pragma unroll 1
        for (int st = 0; st < 4; ++st) {
            kite_rhs<DT, WIND>(P, xs, u, kv, WIND ? wind + 3 * b : nullptr);
            const ST wa = (st == 0 || st == 3) ? hs / ST(6) : hs / ST(3);
            const ST wn = (st < 2) ? ST(0.5) * hs : hs;
#pragma unroll
            for (int i = 0; i < NK; ++i) {
                acc[i] = rk_axpy<DT, ST>(wa, kv[i], acc[i]);
                xs[i] = rk_axpy<DT, ST>(wn, kv[i], x[i]);
            }
        }
#pragma unroll
        for (int i = 0; i < NK; ++i) x[i] = acc[i];
    }
    double* ab = AB + ((size_t)b * N + k) * (NK * 16);
#pragma unroll
    for (int i = 0; i < NK; ++i) {
        ab[i * 16 + d0] = (double)x[i].a;
        ab[i * 16 + d1] = (double)x[i].b;
    }
    if constexpr (std::is_same<ST, double>::value) {
        if (d == 0) {
            const double* xn = X + ((size_t)b * (N + 1) + k + 1) * NX;
            double* df = DEF + ((size_t)b * N + k) * NK;
#pragma unroll
            for (int i = 0; i < NK; ++i) df[i] = x[i].v - xn[i];
        }
    }
}

// Latency form for small batches (B <= RK1_MAXB, fp64): ONE tangent per lane,
// 16 lanes per (instance, interval), four instances per 64-thread block.
// Each lane runs about 60 % of a Dual2 lane's instructions, so a batch too
// small to fill the GPU (one kite: 20 intervals) finishes its RK4 chains
// sooner; at large batches the Dual2 form's shared primal wins.
// Same per-direction arithmetic as Dual2 (the operators are written alike).
constexpr int RK1_T = 64, RK1_MAXB = 128;
__global__ __launch_bounds__(RK1_T, 1) void k_rk4_sens1(ModelConst P, int B, int N, int M, double h,
                                                        const double* __restrict__ X,
                                                        const double* __restrict__ U,
                                                        double* __restrict__ AB, double* __restrict__ DEF) {
    const int d = threadIdx.x & 15;
    const int b = blockIdx.x * (RK1_T / 16) + (threadIdx.x >> 4);
    const int k = blockIdx.y;
    if (b >= B) return;
    const double* xk = X + ((size_t)b * (N + 1) + k) * NX;
    const double* uk = U + ((size_t)b * N + k) * NU;
    Dual x[NK], u[NKU];
#pragma unroll
    for (int i = 0; i < NK; ++i) x[i] = Dual(xk[i], d == i ? 1.0 : 0.0);
#pragma unroll
    for (int j = 0; j < NKU; ++j) u[j] = Dual(uk[j], d == NK + j ? 1.0 : 0.0);
#pragma unroll 1
    for (int m = 0; m < M; ++m) {
        Dual xs[NK], acc[NK], kv[NK];
#pragma unroll
        for (int i = 0; i < NK; ++i) { xs[i] = x[i]; acc[i] = x[i]; }
#pragma unroll 1
        for (int st = 0; st < 4; ++st) {
            kite_rhs<Dual, false>(P, xs, u, kv, nullptr);
            const double wa = (st == 0 || st == 3) ? h / 6.0 : h / 3.0;
            const double wn = (st < 2) ? 0.5 * h : h;
#pragma unroll
            for (int i = 0; i < NK; ++i) {
                acc[i] = Dual(fma(wa, kv[i].v, acc[i].v), fma(wa, kv[i].t, acc[i].t));
                xs[i] = Dual(fma(wn, kv[i].v, x[i].v), fma(wn, kv[i].t, x[i].t));
            }
        }
#pragma unroll
        for (int i = 0; i < NK; ++i) x[i] = acc[i];
    }
    double* ab = AB + ((size_t)b * N + k) * (NK * 16);
#pragma unroll
    for (int i = 0; i < NK; ++i) ab[i * 16 + d] = x[i].t;
    if (d == 0) {
        const double* xn = X + ((size_t)b * (N + 1) + k + 1) * NX;
        double* df = DEF + ((size_t)b * N + k) * NK;
#pragma unroll
        for (int i = 0; i < NK; ++i) df[i] = x[i].v - xn[i];
    }
}

// fp64 multiple-shooting defects x+(x_k, u_k) - x_{k+1}, lane per (instance,
// interval): the right-hand side of the QP when the sensitivities run in fp32
__global__ __launch_bounds__(64, 2) void k_defects(ModelConst P, int B, int N, int M, double h,
                                                 const double* __restrict__ X, const double* __restrict__ U,
                                                 double* __restrict__ DEF, const double* __restrict__ wind) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= B * N) return;
    const int b = g / N, k = g % N;
    const double* xk = X + ((size_t)b * (N + 1) + k) * NX;
    const double* uk = U + ((size_t)b * N + k) * NU;
    double x0[NX], u4[NU], xo[NX];
    for (int i = 0; i < NX; ++i) x0[i] = xk[i];
    for (int j = 0; j < NU; ++j) u4[j] = uk[j];
    if (wind) rk4_primal<true>(P, x0, u4, h, M, xo, wind + 3 * b);
    else rk4_primal(P, x0, u4, h, M, xo);
    double* df = DEF + ((size_t)b * N + k) * NK;
    for (int i = 0; i < NK; ++i) df[i] = xo[i] - xk[NX + i];
}

// ---------------------------------------------------------------------------
// k_condense: one wavefront per instance.
//   lane j < 3N  : column j of G (kite control (k=j/3, c=j%3)), 13 rows in VGPRs
//   lane 3N      : affine column g (propagated defects)
// Per node k the lanes write the Gauss-Newton residual rows W_k (3 path rows,
// 1 path-speed row) into a 16-row LDS chunk; every 4 nodes the chunk is
// folded into H_ext = W_ext^T W_ext (96 x 96, 21 lower 16x16 tiles held in
// MFMA accumulators) with v_mfma_f64_16x16x4_f64.  Column n of W_ext is the
// residual value, so H_ext[n][:] is the gradient.
// ---------------------------------------------------------------------------
constexpr int QP_NTA = 5;       // tiled QP: control block 4N = 80 = 5 tiles (N = 20)
constexpr int QP_NTILE = QP_NTA * (QP_NTA + 1) / 2;   // 15 lower tiles


__device__ __forceinline__ double col_scale(const RtiConst& C, int j) {
    const int N = C.N;
    if (j < 3 * N) return 1.0 / C.Su[j % 3];
    if (j < 4 * N) return 1.0 / C.Su[3];
    if (j == 4 * N) return 1.0 / C.Sx13;
    return 1.0 / C.Sx14;
}
__device__ __forceinline__ double col_rdiag(const RtiConst& C, int j) {
    const int N = C.N;
    if (j < 3 * N) return C.Rdiag[j % 3];
    if (j < 4 * N) return C.Rdiag[3];
    return 0.0;
}
// the per-column scaling constants in registers (select-indexed: no dynamic
// indexing into the kernel-argument struct, which would copy it to scratch)
struct ColConst {
    int N;
    double iSu0, iSu1, iSu2, iSu3, iSx13, iSx14, Rd0, Rd1, Rd2, Rd3;
};
__device__ __forceinline__ ColConst col_const(const RtiConst& C) {
    return ColConst{C.N, 1.0 / C.Su[0], 1.0 / C.Su[1], 1.0 / C.Su[2], 1.0 / C.Su[3], 1.0 / C.Sx13, 1.0 / C.Sx14,
                    C.Rdiag[0], C.Rdiag[1], C.Rdiag[2], C.Rdiag[3]};
}
__device__ __forceinline__ double col_scale(const ColConst& K, int j) {
    if (j < 3 * K.N) { const int c = j % 3; return c == 0 ? K.iSu0 : (c == 1 ? K.iSu1 : K.iSu2); }
    if (j < 4 * K.N) return K.iSu3;
    return j == 4 * K.N ? K.iSx13 : K.iSx14;
}
__device__ __forceinline__ double col_rdiag(const ColConst& K, int j) {
    if (j < 3 * K.N) { const int c = j % 3; return c == 0 ? K.Rd0 : (c == 1 ? K.Rd1 : K.Rd2); }
    if (j < 4 * K.N) return K.Rd3;
    return 0.0;
}
__device__ __forceinline__ double col_ubar(const RtiConst& C, const double* Ub, int j) {
    const int N = C.N;
    if (j < 3 * N) return Ub[(j / 3) * NU + (j % 3)];
    if (j < 4 * N) return Ub[(j - 3 * N) * NU + 3];
    return 0.0;
}

// Condensing kernel, NW = 1..4 wavefronts per instance (CondenseGeom).
//   threads t < 3N : column t of G (kite control (k=t/3, c=t%3)), 13 rows in VGPRs
//   thread  3N     : affine column g (propagated defects)
//   wave w         : MFMA accumulators of the lower tiles in its tile-row range
//                    of H_ext (NR = ceil((n+1)/16) rows, balanced tile counts)
// The affine column's values are shared through LDS (sG), the 16-row W chunk
// (4 nodes) through LDS; every wave folds each chunk into its own tiles.
template <int NR>
struct CondenseGeom {
    static constexpr int T = NR * (NR + 1) / 2;                        // lower tiles of H_ext
    static constexpr int NW = T <= 10 ? 1 : ((T + 11) / 12 > 4 ? 4 : (T + 11) / 12);   // waves per instance
    // first tile row of wave w: the row boundary whose tile count is closest
    // to w T / NW (balances the accumulators of the waves)
    static constexpr int lo(int w) {
        if (w <= 0) return 0;
        if (w >= NW) return NR;
        int best = 0;
        for (int r = 1; r < NR; ++r) {
            const int d0 = 2 * NW * (r * (r + 1) / 2) - 2 * w * T;
            const int d1 = 2 * NW * (best * (best + 1) / 2) - 2 * w * T;
            if ((d0 < 0 ? -d0 : d0) < (d1 < 0 ? -d1 : d1)) best = r;
        }
        return best < lo(w - 1) ? lo(w - 1) : best;
    }
    static constexpr int tiles(int w) { return (lo(w + 1) * (lo(w + 1) + 1) - lo(w) * (lo(w) + 1)) / 2; }
    static constexpr int acc() {
        int m = 1;
        for (int w = 0; w < NW; ++w) m = tiles(w) > m ? tiles(w) : m;
        return m;
    }
    static constexpr int ACC = acc();
    static constexpr int WLD = 16 * NR + ((NR % 2 == 0) ? 16 : 32);   // 2*WLD % 64 == 32: conflict-free
};

// Per-wave tile loops with compile-time tile coordinates: wave W owns the
// lower tiles (I, J <= I) of tile rows [lo(W), lo(W+1)), accumulator slot Q.
template <int NR, int W, int I, int J, int Q>
__device__ __forceinline__ void fold_rec(double4v* acc, const double* fr) {
    if constexpr (I < CondenseGeom<NR>::lo(W + 1)) {
        acc[Q] = __builtin_amdgcn_mfma_f64_16x16x4f64(fr[I], fr[J], acc[Q], 0, 0, 0);
        if constexpr (J < I) fold_rec<NR, W, I, J + 1, Q + 1>(acc, fr);
        else fold_rec<NR, W, I + 1, 0, Q + 1>(acc, fr);
    }
}
template <int NR, int W>
__device__ __forceinline__ void wave_fold(int w, double4v* acc, const double* fr) {
    if (w == W) fold_rec<NR, W, CondenseGeom<NR>::lo(W), 0, 0>(acc, fr);
    else if constexpr (W + 1 < CondenseGeom<NR>::NW) wave_fold<NR, W + 1>(w, acc, fr);
}
template <int NR, int W, int I, int J, int Q, class F>
__device__ __forceinline__ void put_rec(const double4v* acc, F& put) {
    if constexpr (I < CondenseGeom<NR>::lo(W + 1)) {
        put(I, J, acc[Q]);
        if constexpr (J < I) put_rec<NR, W, I, J + 1, Q + 1>(acc, put);
        else put_rec<NR, W, I + 1, 0, Q + 1>(acc, put);
    }
}
template <int NR, int W, class F>
__device__ __forceinline__ void wave_put(int w, const double4v* acc, F& put) {
    if (w == W) put_rec<NR, W, CondenseGeom<NR>::lo(W), 0, 0>(acc, put);
    else if constexpr (W + 1 < CondenseGeom<NR>::NW) wave_put<NR, W + 1>(w, acc, put);
}

// Optional phase profile of k_condense (-DKITE_QP_PROF, tools only): shader
// clock cycles of wave 0 per phase, summed over instances into g_cd_prof.
#ifdef KITE_QP_PROF
__device__ unsigned long long g_cd_prof[8];
#define CD_MARK(ph)                                                                  \
    do {                                                                             \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                  \
        cd_acc[ph] += t_ - cd_last;                                                  \
        cd_last = t_;                                                                \
    } while (0)
#else
#define CD_MARK(ph) do { } while (0)
#endif

template <int NR>
__global__ __launch_bounds__(64 * CondenseGeom<NR>::NW) __attribute__((amdgpu_waves_per_eu(NR <= 7 ? 2 : 1))) void k_condense(RtiConst C, int B, const double* __restrict__ X,
                                                  const double* __restrict__ U, const double* __restrict__ AB,
                                                  const double* __restrict__ DEF, double* __restrict__ Hs,
                                                  double* __restrict__ hs, double* __restrict__ Cr,
                                                  double* __restrict__ cl, double* __restrict__ cu,
                                                  double* __restrict__ hmax, int tiled, double* __restrict__ Htl,
                                                  double* __restrict__ Hab, double* __restrict__ Hbb) {
    using Gm = CondenseGeom<NR>;
    constexpr int WLDc = Gm::WLD;
    constexpr int NT = 64 * Gm::NW;
    constexpr int NMAX = (16 * NR - 3) / 4;          // largest horizon with n + 1 <= 16 NR
    constexpr int SAL = 16 * 16 + NK + 3;
    __shared__ double sA[2][SAL];                    // [A_k | B_k] by columns (col j: 16 j + i), then d_k;
                                                     // double-buffered by node parity
    __shared__ double Wc[16 * WLDc];
    __shared__ double sG[2][4];                      // affine column rows 0, 6..8, by node parity
    __shared__ double sX[(NMAX + 1) * NX];           // linearisation trajectory
    __shared__ double sPth[NMAX + 1][6];             // P(theta_k), dP/dtheta(theta_k)
    // vx-bound rows on the kite controls, staged for one bulk store after the
    // node loop (short horizons; the long ones keep per-node stores: LDS)
    constexpr bool STAGE_C = NR <= 6;           // LDS <= 38 KB: still 4 blocks per CU
    constexpr int CLD = 3 * NMAX;
    __shared__ double sCr[STAGE_C ? NMAX * CLD : 1];
    __shared__ double sCl[STAGE_C ? NMAX : 1], sCu[STAGE_C ? NMAX : 1];
    __shared__ double sMax[4];
    // per-variable column scaling D, R diagonal and R ubar of the output
    // stage (a table: lane-dependent selects over kernel-argument fields
    // would be lowered to scratch)
    __shared__ double sScl[16 * NR], sRd[16 * NR], sRu[16 * NR];
#ifdef KITE_QP_PROF
    unsigned long long cd_acc[6] = {0, 0, 0, 0, 0, 0};
    unsigned long long cd_last = __builtin_amdgcn_s_memtime();
#endif
    const int b = blockIdx.x;
    const int t = threadIdx.x;
    const int l = t & 63, w = t >> 6;
    const int N = C.N, n = C.n;
    const double* Xb = X + (size_t)b * (N + 1) * NX;
    const double* Ub = U + (size_t)b * N * NU;
    const double* ABb = AB + (size_t)b * N * NK * 16;
    const double* DEFb = DEF + (size_t)b * N * NK;

    for (int i = t; i < 16 * WLDc; i += NT) Wc[i] = 0.0;
    if (t < 8) sG[t >> 2][t & 3] = 0.0;
    // the trajectory and the path at every node up front (lane per node): the
    // node loop below is a dependent chain and reads both from LDS only
    {
        constexpr int NXL = ((NMAX + 1) * NX + NT - 1) / NT;    // loads per thread, all in flight
        double xv[NXL];
#pragma unroll
        for (int q = 0; q < NXL; ++q) {
            const int i = t + NT * q;
            xv[q] = i < (N + 1) * NX ? Xb[i] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < NXL; ++q) {
            const int i = t + NT * q;
            if (i < (N + 1) * NX) sX[i] = xv[q];
        }
    }
    if (t <= N) {
        double Pp[3], dP[3];
        path_eval(C, Xb[t * NX + 13], Pp, dP);
#pragma unroll
        for (int a = 0; a < 3; ++a) { sPth[t][a] = Pp[a]; sPth[t][3 + a] = dP[a]; }
    }
    {
        const double iS0 = 1.0 / C.Su[0], iS1 = 1.0 / C.Su[1], iS2 = 1.0 / C.Su[2], iS3 = 1.0 / C.Su[3];
        const double R0 = C.Rdiag[0], R1 = C.Rdiag[1], R2 = C.Rdiag[2], R3 = C.Rdiag[3];
        for (int i = t; i < 16 * NR; i += NT) {
            double sc = 0.0, rd = 0.0, ub = 0.0;
            if (i < 3 * N) {
                const int c = i % 3;
                sc = c == 0 ? iS0 : (c == 1 ? iS1 : iS2);
                rd = c == 0 ? R0 : (c == 1 ? R1 : R2);
                ub = Ub[(i / 3) * NU + c];
            } else if (i < 4 * N) {
                sc = iS3; rd = R3; ub = Ub[(i - 3 * N) * NU + 3];
            } else if (i == 4 * N) {
                sc = 1.0 / C.Sx13;
            } else if (i == 4 * N + 1) {
                sc = 1.0 / C.Sx14;
            }
            sScl[i] = sc; sRd[i] = rd; sRu[i] = rd * ub;
        }
    }

    const bool kite_lane = t < 3 * N;
    const bool aff_lane = (t == 3 * N);
    const int kb = t / 3, cc = t % 3;
    const double Dl = kite_lane ? 1.0 / C.Su[cc] : 0.0;
    double v[NK];
#pragma unroll
    for (int i = 0; i < NK; ++i) v[i] = 0.0;

    double4v acc[Gm::ACC];
#pragma unroll
    for (int q = 0; q < Gm::ACC; ++q) acc[q] = double4v{0.0, 0.0, 0.0, 0.0};

    // software prefetch of the interval data (221 doubles -> <= 2 per thread),
    // PD intervals ahead in a register ring: the node loop is a dependent
    // chain, so one interval of look-ahead would expose the global latency
    constexpr int NPF = (NK * 16 + NK + NT - 1) / NT;
    constexpr int PD = 2;
    double pf[PD][NPF];
    auto load_iv = [&](int k, double* dst) __attribute__((always_inline)) {
#pragma unroll
        for (int q = 0; q < NPF; ++q) {
            const int e = t + NT * q;
            double val = 0.0;
            if (e < NK * 16) val = ABb[(size_t)k * NK * 16 + e];
            else if (e < NK * 16 + NK) val = DEFb[(size_t)k * NK + (e - NK * 16)];
            dst[q] = val;
        }
    };
#pragma unroll
    for (int s = 0; s < PD; ++s)
        if (s < N) load_iv(s, pf[s]);
    __syncthreads();

    // residual row weights in registers: stage sqrt(dt Q) Sr, Mayer sqrt(Q) Sr
    double wpD[3], wpT[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) { wpD[a] = C.sqQ_dt[a] * C.Sr[a]; wpT[a] = C.sqQ_T[a] * C.Sr[a]; }
    // Node loop, one barrier per node: sA and sG are double-buffered by node
    // parity, so the barrier that publishes interval k also orders the affine
    // values of node k (written after the previous barrier) and the previous
    // chunk fold before this node's W rows overwrite Wc.
    CD_MARK(0);
    auto node = [&](int k, double* pfs) __attribute__((always_inline)) {
        const bool last = (k == N);
        const int par = k & 1;
        if (!last) {
#pragma unroll
            for (int q = 0; q < NPF; ++q) {
                const int e = t + NT * q;
                if (e < NK * 16) sA[par][(e & 15) * 16 + (e >> 4)] = pfs[q];      // transpose: column-major
                else if (e < NK * 16 + NK) sA[par][16 * 16 + (e - NK * 16)] = pfs[q];
            }
        }
        __syncthreads();
        CD_MARK(1);
        if (k + PD < N) load_iv(k + PD, pfs);
        const double* xk = sX + k * NX;
        const double thd = xk[14];
        const double Pp[3] = {sPth[k][0], sPth[k][1], sPth[k][2]};
        const double dP[3] = {sPth[k][3], sPth[k][4], sPth[k][5]};
        const double g0 = sG[par ^ 1][0];
        const double gr[3] = {sG[par ^ 1][1], sG[par ^ 1][2], sG[par ^ 1][3]};
        double wp[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) wp[a] = last ? wpT[a] : wpD[a];
        const double wv = last ? 0.0 : C.sw * C.sv;
        const int row0 = 4 * (k & 3);

        // kite columns: path rows -sq sr G[6+a], speed row 0
        if (kite_lane) {
            Wc[(row0 + 0) * WLDc + t] = -wp[0] * v[6];
            Wc[(row0 + 1) * WLDc + t] = -wp[1] * v[7];
            Wc[(row0 + 2) * WLDc + t] = -wp[2] * v[8];
            Wc[(row0 + 3) * WLDc + t] = 0.0;
        }
        // analytic columns 3N .. n (Uv_m, theta0, thetadot0, affine)
        if (t < N + 3) {
            const int col = 3 * N + t;
            double cth = 0.0, cthd = 0.0;
            if (t < N) {
                if (k > t) { cth = C.dt * C.dt * ((double)(k - t) - 0.5); cthd = C.dt; }
            } else if (t == N) {
                cth = 1.0;
            } else if (t == N + 1) {
                cth = (double)k * C.dt; cthd = 1.0;
            }
            if (t < N + 2) {
#pragma unroll
                for (int a = 0; a < 3; ++a) Wc[(row0 + a) * WLDc + col] = wp[a] * dP[a] * cth;
                Wc[(row0 + 3) * WLDc + col] = -wv * cthd;
            } else {
#pragma unroll
                for (int a = 0; a < 3; ++a) Wc[(row0 + a) * WLDc + col] = wp[a] * (Pp[a] - xk[6 + a] - gr[a]);
                Wc[(row0 + 3) * WLDc + col] = last ? 0.0 : C.sw * (C.sv * C.vref - C.sv * thd);
            }
        }
        // vx bound rows (node k >= 1)
        if (k >= 1) {
            const double cv = v[0] * Dl;
            const double base = xk[0] + g0;
            const double clv = C.lo_fin ? (C.lbx[0] - base) : -INFINITY;
            const double cuv = C.hi_fin ? (C.ubx[0] - base) : INFINITY;
            if constexpr (STAGE_C) {
                if (kite_lane) sCr[(k - 1) * CLD + t] = cv;
                if (t == 0) { sCl[k - 1] = clv; sCu[k - 1] = cuv; }
            } else {
                double* crow = Cr + ((size_t)b * N + (k - 1)) * n;
                if (kite_lane) crow[t] = cv;
                if (t < N + 2) crow[3 * N + t] = 0.0;
                if (t == 0) { cl[(size_t)b * N + k - 1] = clv; cu[(size_t)b * N + k - 1] = cuv; }
            }
        }
        if (last) {
            // zero the rows of nodes beyond N in this chunk
            for (int r = row0 + 4; r < 16; ++r)
                for (int cidx = t; cidx <= n; cidx += NT) Wc[r * WLDc + cidx] = 0.0;
        }
        CD_MARK(2);
        if (!last) {
            // propagate G_{k+1} = A_k G_k (+ B_k e_c at k == kb), g_{k+1} = A_k g_k + d_k
            const double* sa = sA[par];
            if ((kite_lane && k >= kb) || aff_lane) {
                double nv[NK];
                if (kite_lane && k == kb) {
#pragma unroll
                    for (int i = 0; i < NK; ++i) nv[i] = sa[(NK + cc) * 16 + i];
                } else {
                    // column-oriented: 13 independent accumulator chains, the
                    // next column's loads in flight under this column's FMAs
                    const double am = aff_lane ? 1.0 : 0.0;
#pragma unroll
                    for (int i = 0; i < NK; ++i) nv[i] = am * sa[16 * 16 + i];
                    double ac[NK], an[NK];
#pragma unroll
                    for (int i = 0; i < NK; ++i) ac[i] = sa[i];
#pragma unroll
                    for (int j = 0; j < NK; ++j) {
                        if (j + 1 < NK) {
#pragma unroll
                            for (int i = 0; i < NK; ++i) an[i] = sa[(j + 1) * 16 + i];
                        }
#pragma unroll
                        for (int i = 0; i < NK; ++i) nv[i] = fma(ac[i], v[j], nv[i]);
                        asm volatile("s_nop 0" ::: "memory");   // at most two columns of A_k in registers
#pragma unroll
                        for (int i = 0; i < NK; ++i) ac[i] = an[i];
                    }
                }
#pragma unroll
                for (int i = 0; i < NK; ++i) v[i] = nv[i];
            }
            if (aff_lane) { sG[par][0] = v[0]; sG[par][1] = v[6]; sG[par][2] = v[7]; sG[par][3] = v[8]; }
        }
        CD_MARK(3);
        if ((k & 3) == 3 || last) {
            __syncthreads();
            // fold the chunk: every wave into the tiles of its own tile rows
            // (the next node's barrier orders these reads before Wc is rewritten)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                double fr[NR];
#pragma unroll
                for (int I = 0; I < NR; ++I) fr[I] = Wc[(4 * s + (l >> 4)) * WLDc + 16 * I + (l & 15)];
                wave_fold<NR, 0>(w, acc, fr);
            }
            CD_MARK(4);
        }
    };
#pragma unroll 1
    for (int k0 = 0; k0 <= N; k0 += PD) {
        node(k0, pf[0]);
        if (k0 + 1 > N) break;
        node(k0 + 1, pf[1]);
    }
    __syncthreads();

    // vx-bound rows C (kite-control columns from sCr, the rest zero) and their bounds
    if constexpr (STAGE_C) {
        for (int e = t; e < N * n; e += NT) {
            const int r = e / n, c = e % n;
            Cr[(size_t)b * N * n + e] = c < 3 * N ? sCr[r * CLD + c] : 0.0;
        }
        if (t < N) { cl[(size_t)b * N + t] = sCl[t]; cu[(size_t)b * N + t] = sCu[t]; }
    }

    // write the scaled QP: Hs = D (H + Rdiag) D, hs = D (g + Rdiag ubar).
    // tiled != 0 (k_qp_tiled N = 20, k_qp_lds N = 40): the control block H_aa (na = 4N = 16*NT)
    // goes out as C-layout tiles in lane order [tile][reg][lane], the theta
    // couplings as H_ab [na][2] and H_bb [2][2]; otherwise the full n x n H.
    double* Hb = Hs + (size_t)b * n * n;
    const int na = 4 * N;
    const int ntile = (N / 4) * (N / 4 + 1) / 2;       // tiled: lower tiles of H_aa (N % 4 == 0)
    double lmax = 0.0;
    auto put = [&](int I, int J, double4v a4) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int gi = 16 * I + (l >> 4) + 4 * r;
            const int gj = 16 * J + (l & 15);
            const double a = a4[r];
            if (gi < n && gj < n) {
                double hv = a;
                if (gi == gj) hv += sRd[gi];
                hv *= sScl[gi] * sScl[gj];
                if (tiled) {
                    if (gi < na) Htl[((size_t)b * ntile + I * (I + 1) / 2 + J) * 256 + r * 64 + l] = hv;
                    else if (gj < na) Hab[((size_t)b * na + gj) * 2 + (gi - na)] = hv;
                    else {
                        Hbb[(size_t)b * 4 + (gi - na) * 2 + (gj - na)] = hv;
                        Hbb[(size_t)b * 4 + (gj - na) * 2 + (gi - na)] = hv;
                    }
                } else {
                    Hb[(size_t)gi * n + gj] = hv;
                    Hb[(size_t)gj * n + gi] = hv;
                }
                lmax = fmax(lmax, fabs(hv));
            } else if (gi == n && gj < n) {
                hs[(size_t)b * n + gj] = (a + sRu[gj]) * sScl[gj];
            }
        }
    };
    wave_put<NR, 0>(w, acc, put);
    lmax = wave_max(lmax);
    if (l == 0) sMax[w] = lmax;
    __syncthreads();
    if (t == 0) {
        double m = sMax[0];
        for (int i = 1; i < Gm::NW; ++i) m = fmax(m, sMax[i]);
        hmax[b] = m;
    }
#ifdef KITE_QP_PROF
    CD_MARK(5);
    if (t == 0) {
        for (int i = 0; i < 6; ++i) atomicAdd(&g_cd_prof[i], cd_acc[i]);
        atomicAdd(&g_cd_prof[7], 1ull);
    }
#endif
}

// ---------------------------------------------------------------------------
// k_condense20: N = 20 condensing for the tiled QP, ONE wavefront per kite.
// Same algebra as k_condense, organised for latency: every node's 4 residual
// rows (3 path rows, 1 path-speed row; Mayer rows at node N) ARE one k-step
// of v_mfma_f64_16x16x4_f64, so each node is folded into H_aa as soon as its
// rows exist (15 lower 16x16 tiles = 60 accumulators per lane) -- no 16-row
// chunk buffer, no second wave, no block barrier (wavefront fences only).
// The three columns past the control block (theta0, thetadot0 and the
// affine residual column that yields the gradient) are accumulated on the
// VALU against variable i = l (slot 0) and 64 + l (slot 1): H_ab, H_bb and h
// come straight out of them.  Small footprint (~10 KB LDS) so two kites share
// a SIMD (launch bound 2 waves / SIMD).
//   lane t < 60 : column t of G (kite control (k = t/3, c = t%3)), 13 rows in VGPRs
//   lane 60     : the affine column g (propagated defects)
// The propagation G_{k+1} = A_k G_k needs every element of A_k in every lane.
// Round 5 moved it from LDS broadcast reads (169 ds_read_b64 per node and
// kite, 86 KB of LDS return traffic: the CU's LDS was the kernel's bound) to
// register-resident columns broadcast inside the FMA (fmac_col13): 0.184 ->
// 0.140 ms, bitwise the same output (profiles/r05l_condense_dpp_ab.txt).
// ---------------------------------------------------------------------------
// nv[i] += A[i][j] * v_j for the 13 rows i of one column j, the column held in
// ONE register in row layout (lane p of every 16-lane row holds A[p][j]):
// v_fmac_f64_dpp with row_newbcast:i broadcasts A[i][j] to the whole row
// inside the FMA -- no LDS broadcast read.  The compiler does not form this
// instruction itself (it keeps a v_mov_b64_dpp + v_fmac_f64 pair), and its
// hazard recognizer does not look into inline asm: the leading s_nop 1 covers
// the two wait states a VALU write of the DPP source needs (the column comes
// from a global load, but the register allocator may copy it), and the
// trailing s_nop 1 the two a DPP / permlane after the block needs if it reads
// an nv register the last fmac wrote.  Every lane of a row needs the
// broadcast, so the block is correct only with the full EXEC mask:
// k_condense20 calls it only under the wave-uniform `!last` (64-lane blocks,
// no divergent branch around it).
#define KITE_FMAC_DPP(I) "v_fmac_f64_dpp %" #I ", %13, %14 row_newbcast:" #I " row_mask:0xf bank_mask:0xf\n\t"
__device__ __forceinline__ void fmac_col13(double (&nv)[NK], double a, double vj) {
    asm("s_nop 1\n\t"
        KITE_FMAC_DPP(0) KITE_FMAC_DPP(1) KITE_FMAC_DPP(2) KITE_FMAC_DPP(3) KITE_FMAC_DPP(4)
        KITE_FMAC_DPP(5) KITE_FMAC_DPP(6) KITE_FMAC_DPP(7) KITE_FMAC_DPP(8) KITE_FMAC_DPP(9)
        KITE_FMAC_DPP(10) KITE_FMAC_DPP(11) KITE_FMAC_DPP(12) "s_nop 1"
        : "+v"(nv[0]), "+v"(nv[1]), "+v"(nv[2]), "+v"(nv[3]), "+v"(nv[4]), "+v"(nv[5]), "+v"(nv[6]),
          "+v"(nv[7]), "+v"(nv[8]), "+v"(nv[9]), "+v"(nv[10]), "+v"(nv[11]), "+v"(nv[12])
        : "v"(a), "v"(vj));
}
#undef KITE_FMAC_DPP

constexpr int CD20_N = 20, CD20_NA = 80, CD20_n = 82;
constexpr int CD20_WLD = 112;                    // Wc row stride: 2*WLD % 64 == 32 -> conflict-free tile reads
__global__ __launch_bounds__(64, 2) void k_condense20(RtiConst C, int B, const double* __restrict__ X,
                                                      const double* __restrict__ U,
                                                      const double* __restrict__ AB,
                                                      const double* __restrict__ DEF, double* __restrict__ hs,
                                                      double* __restrict__ Cr, double* __restrict__ cl,
                                                      double* __restrict__ cu, double* __restrict__ hmax,
                                                      double* __restrict__ Htl, double* __restrict__ Hab,
                                                      double* __restrict__ Hbb) {
    constexpr int N = CD20_N, n = CD20_n, NA = CD20_NA, WLD = CD20_WLD;
    __shared__ double Wc[4 * WLD];                   // the 4 residual rows of the current node
    __shared__ double sX[(N + 1) * NX];
    __shared__ double sPth[N + 1][6];
    __shared__ double sScl[96], sRd[96], sRu[96];
    __shared__ double sHx[3][96];
    const int b = blockIdx.x;
    const int l = threadIdx.x;
    if (b >= B) return;
    const double* Xb = X + (size_t)b * (N + 1) * NX;
    const double* Ub = U + (size_t)b * N * NU;
    const double* ABb = AB + (size_t)b * N * NK * 16;
    const double* DEFb = DEF + (size_t)b * N * NK;

    {   // trajectory up front (all loads in flight first), path per node, scale tables
        constexpr int NXL = ((N + 1) * NX + 63) / 64;
        double xv[NXL];
#pragma unroll
        for (int q = 0; q < NXL; ++q) {
            const int i = l + 64 * q;
            xv[q] = i < (N + 1) * NX ? Xb[i] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < NXL; ++q) {
            const int i = l + 64 * q;
            if (i < (N + 1) * NX) sX[i] = xv[q];
        }
    }
    if (l <= N) {
        double Pp[3], dP[3];
        path_eval(C, Xb[l * NX + 13], Pp, dP);
#pragma unroll
        for (int a = 0; a < 3; ++a) { sPth[l][a] = Pp[a]; sPth[l][3 + a] = dP[a]; }
    }
    {
        const double iS0 = 1.0 / C.Su[0], iS1 = 1.0 / C.Su[1], iS2 = 1.0 / C.Su[2], iS3 = 1.0 / C.Su[3];
        const double R0 = C.Rdiag[0], R1 = C.Rdiag[1], R2 = C.Rdiag[2], R3 = C.Rdiag[3];
        for (int i = l; i < 96; i += 64) {
            double sc = 0.0, rd = 0.0, ub = 0.0;
            if (i < 3 * N) {
                const int c = i % 3;
                sc = c == 0 ? iS0 : (c == 1 ? iS1 : iS2);
                rd = c == 0 ? R0 : (c == 1 ? R1 : R2);
                ub = Ub[(i / 3) * NU + c];
            } else if (i < 4 * N) {
                sc = iS3; rd = R3; ub = Ub[(i - 3 * N) * NU + 3];
            } else if (i == 4 * N) {
                sc = 1.0 / C.Sx13;
            } else if (i == 4 * N + 1) {
                sc = 1.0 / C.Sx14;
            }
            sScl[i] = sc; sRd[i] = rd; sRu[i] = rd * ub;
        }
    }
    const bool kite_lane = l < 3 * N;
    const bool aff_lane = (l == 3 * N);
    const int kb = l / 3, cc = l % 3;
    // select by value: a lane-dependent index into the kernel-argument struct
    // would copy the struct to scratch
    const double Dl = kite_lane ? 1.0 / (cc == 0 ? C.Su[0] : (cc == 1 ? C.Su[1] : C.Su[2])) : 0.0;
    double v[NK];
#pragma unroll
    for (int i = 0; i < NK; ++i) v[i] = 0.0;
    double4v acc[QP_NTILE];
#pragma unroll
    for (int q = 0; q < QP_NTILE; ++q) acc[q] = double4v{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int c = 0; c < 3; ++c) {                    // H_ext[i][80 + c], i < 83
        sHx[c][l] = 0.0;
        if (l < 96 - 64) sHx[c][64 + l] = 0.0;
    }

    // interval data of the next node in registers, row layout: lane l holds row
    // p = l & 15 of [A_k | B_k] (Ar[j], j < 16) and d_k[p] (Ar[16]); rows 13..15
    // repeat row 12 and are never read (the broadcasts take lanes 0..12).  Loaded
    // right after the previous node's propagation, consumed by the next one: the
    // node's fold runs in between.
    typedef double double2v __attribute__((ext_vector_type(2)));
    double Ar[16 + 1];
    auto load_ar = [&](int k) __attribute__((always_inline)) {
        const int p = min(l & 15, NK - 1);
        const double2v* src = reinterpret_cast<const double2v*>(ABb + (size_t)k * NK * 16 + (size_t)p * 16);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const double2v t2 = src[q];
            Ar[2 * q] = t2[0];
            Ar[2 * q + 1] = t2[1];
        }
        Ar[16] = DEFb[(size_t)k * NK + p];
    };
    load_ar(0);
    double wpD[3], wpT[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) { wpD[a] = C.sqQ_dt[a] * C.Sr[a]; wpT[a] = C.sqQ_T[a] * C.Sr[a]; }
    double* Crb = Cr + (size_t)b * N * n;

    auto node = [&](int k) __attribute__((always_inline)) {
        const bool last = (k == N);
        wave_sync();                  // the previous node's Wc reads are done
        // the affine column at node k, wave-uniform (lane 60)
        const double g0 = uniform_d(readlane_d(v[0], 3 * N));
        const double gr0 = uniform_d(readlane_d(v[6], 3 * N));
        const double gr1 = uniform_d(readlane_d(v[7], 3 * N));
        const double gr2 = uniform_d(readlane_d(v[8], 3 * N));
        const double gr[3] = {gr0, gr1, gr2};
        const double* xk = sX + k * NX;
        const double thd = xk[14];
        double wp[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) wp[a] = last ? wpT[a] : wpD[a];
        const double wv = last ? 0.0 : C.sw * C.sv;
        // residual rows of node k: kite columns (path rows -sq sr G[6+a], speed row 0)
        if (kite_lane) {
            Wc[0 * WLD + l] = -wp[0] * v[6];
            Wc[1 * WLD + l] = -wp[1] * v[7];
            Wc[2 * WLD + l] = -wp[2] * v[8];
            Wc[3 * WLD + l] = 0.0;
        }
        // analytic columns 3N .. n (Uv_m, theta0, thetadot0, affine)
        if (l < N + 3) {
            const int col = 3 * N + l;
            double cth = 0.0, cthd = 0.0;
            if (l < N) {
                if (k > l) { cth = C.dt * C.dt * ((double)(k - l) - 0.5); cthd = C.dt; }
            } else if (l == N) {
                cth = 1.0;
            } else if (l == N + 1) {
                cth = (double)k * C.dt; cthd = 1.0;
            }
            if (l < N + 2) {
#pragma unroll
                for (int a = 0; a < 3; ++a) Wc[a * WLD + col] = wp[a] * sPth[k][3 + a] * cth;
                Wc[3 * WLD + col] = -wv * cthd;
            } else {
#pragma unroll
                for (int a = 0; a < 3; ++a) Wc[a * WLD + col] = wp[a] * (sPth[k][a] - xk[6 + a] - gr[a]);
                Wc[3 * WLD + col] = last ? 0.0 : C.sw * (C.sv * C.vref - C.sv * thd);
            }
        }
        // vx bound row of node k >= 1 (kite-control columns; the rest zero)
        if (k >= 1) {
            double* crow = Crb + (size_t)(k - 1) * n;
            crow[l] = kite_lane ? v[0] * Dl : 0.0;
            if (l < n - 64) crow[64 + l] = 0.0;
            if (l == 0) {
                const double base = xk[0] + g0;
                cl[(size_t)b * N + k - 1] = C.lo_fin ? (C.lbx[0] - base) : -INFINITY;
                cu[(size_t)b * N + k - 1] = C.hi_fin ? (C.ubx[0] - base) : INFINITY;
            }
        }
        wave_sync();
        // fold: the node's 4 rows are one MFMA k-step of H_aa += W_k' W_k.
        // Node k's rows reach the kite controls and the Uv of intervals < k
        // only, so tile I (columns 16 I .. 16 I + 15) is zero before node
        // kmin(I) = 1, 6, 11, 1, 5 (tile 3 holds Uv_0..3): the k-steps of zero
        // tiles are skipped (uniform branches; the sums are unchanged, the
        // skipped products are exact zeros) -- 218 instead of 315 MFMAs per kite
        {
            constexpr int kmin[QP_NTA] = {1, 6, 11, 1, 5};
            double fr[QP_NTA];
#pragma unroll
            for (int I = 0; I < QP_NTA; ++I) fr[I] = Wc[(l >> 4) * WLD + 16 * I + (l & 15)];
#pragma unroll
            for (int I = 0; I < QP_NTA; ++I)
#pragma unroll
                for (int J = 0; J <= I; ++J)
                    if (k >= kmin[I] && k >= kmin[J])
                        acc[I * (I + 1) / 2 + J] = __builtin_amdgcn_mfma_f64_16x16x4f64(fr[I], fr[J], acc[I * (I + 1) / 2 + J], 0, 0, 0);
        }
        // the columns past the control block against rows i = l, 64 + l,
        // accumulated in LDS (sHx[c][i]: no long-lived registers)
        {
            double t0[3] = {0.0, 0.0, 0.0}, t1[3] = {0.0, 0.0, 0.0};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double w0 = Wc[r * WLD + l];
                const double w1 = l < n + 1 - 64 ? Wc[r * WLD + 64 + l] : 0.0;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const double we = Wc[r * WLD + NA + c];
                    t0[c] = fma(w0, we, t0[c]);
                    t1[c] = fma(w1, we, t1[c]);
                }
            }
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                sHx[c][l] += t0[c];
                if (l < n + 1 - 64) sHx[c][64 + l] += t1[c];
            }
        }
        if (!last) {
            // G_{k+1} = A_k G_k (+ B_k e_c at k == kb), g_{k+1} = A_k g_k + d_k as
            // one product [A_k | B_k | d_k] [v; e_c at k == kb; 1 on the affine
            // lane], every lane (DPP needs the whole wave; a lane before its
            // start node has v = 0 and stays at +0).  Same terms in the same
            // order as round 4's LDS form (d first, then A column by column;
            // the B terms add exact zeros except at k == kb, where v = 0 and
            // the B column is the value): bitwise the same up to signed zeros.
            double nv[NK];
#pragma unroll
            for (int i = 0; i < NK; ++i) nv[i] = 0.0;
            const bool start = kite_lane && k == kb;
            fmac_col13(nv, Ar[16], aff_lane ? 1.0 : 0.0);
#pragma unroll
            for (int j = 0; j < NK; ++j) fmac_col13(nv, Ar[j], v[j]);
#pragma unroll
            for (int c = 0; c < NKU; ++c) fmac_col13(nv, Ar[NK + c], (start && cc == c) ? 1.0 : 0.0);
#pragma unroll
            for (int i = 0; i < NK; ++i) v[i] = nv[i];
            if (k + 1 < N) load_ar(k + 1);
        }
    };
#pragma unroll 1
    for (int k = 0; k <= N; ++k) node(k);

    // scaled QP out: H_aa tiles (+ R diagonal) in the tiled QP's lane order,
    // H_ab / H_bb / h from the three extra columns; hmax = max |H|
    double lmax = 0.0;
#pragma unroll
    for (int I = 0; I < QP_NTA; ++I)
#pragma unroll
        for (int J = 0; J <= I; ++J) {
            const int t = I * (I + 1) / 2 + J;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gi = 16 * I + (l >> 4) + 4 * r, gj = 16 * J + (l & 15);
                double hv = acc[t][r];
                if (gi == gj) hv += sRd[gi];
                hv *= sScl[gi] * sScl[gj];
                Htl[((size_t)b * QP_NTILE + t) * 256 + r * 64 + l] = hv;
                lmax = fmax(lmax, fabs(hv));
            }
        }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
        const int i = l + 64 * s2;
        const double hxa = i < 96 ? sHx[0][i] : 0.0, hxb = i < 96 ? sHx[1][i] : 0.0;
        const double hxc = i < 96 ? sHx[2][i] : 0.0;
        if (i < NA) {
            const double a0 = hxa * sScl[i] * sScl[NA], a1 = hxb * sScl[i] * sScl[NA + 1];
            Hab[((size_t)b * NA + i) * 2 + 0] = a0;
            Hab[((size_t)b * NA + i) * 2 + 1] = a1;
            lmax = fmax(lmax, fmax(fabs(a0), fabs(a1)));
        } else if (i < n) {
            const double a0 = hxa * sScl[i] * sScl[NA], a1 = hxb * sScl[i] * sScl[NA + 1];
            Hbb[(size_t)b * 4 + (i - NA) * 2 + 0] = a0;
            Hbb[(size_t)b * 4 + (i - NA) * 2 + 1] = a1;
            lmax = fmax(lmax, fmax(fabs(a0), fabs(a1)));
        }
        if (i < n) hs[(size_t)b * n + i] = (hxc + sRu[i]) * sScl[i];
    }
    lmax = wave_max(lmax);
    if (l == 0) hmax[b] = lmax;
}

#ifdef KITE_QP_PROF
// tools only: read and clear the condensing phase profile (8 x uint64)
extern "C" int kite_debug_cd_profile(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_cd_prof), sizeof(g_cd_prof)) != hipSuccess) return -1;
    const unsigned long long z[8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_cd_prof), z, sizeof(z)) != hipSuccess) return -1;
    return 0;
}
#endif

// ---------------------------------------------------------------------------
// k_qp: one wavefront per instance.  Mehrotra predictor-corrector primal-dual
// interior point on
//     min 1/2 w'Hw + h'w   s.t.  lb <= w <= ub,  cl <= C w <= cu
// with a relative freeze (IPM_FREEZE) and cap K, then the expansion
// dx_{k+1} = A_k dx_k + B_k du_k + d_k, the trajectory update, diagnostics
// (kiteNMPF.cpp:319-355) and status.
// The normal matrix is factored in LDS (packed lower triangle).
// ---------------------------------------------------------------------------
// Epilogue of every QP kernel, in two phases so that the state-bound check can
// run on the expanded trajectory BEFORE anything is written (lazy rows):
//   rti_expand : physical step dw = D w into vec[0, n); dx of the kite states
//                (dx_0 = 0, dx_{k+1} = A_k dx_k + B_k du_k + d_k) and the exact
//                theta / thetadot increments into dxs[k * 16 + (0..14)]
//   rti_commit : trajectory and control update, diagnostics
//                (kiteNMPF.cpp:319-355), status.
// One wavefront; w = scaled QP step in slots (i = l + 64 s); vec, dxs: LDS
// scratch (dxs: (N+1) x 16).  WAVE: the LDS exchanges are ordered by a
// wavefront fence, not s_barrier (the caller is one wavefront of a larger
// block).  Returns (wave-uniform) whether the expanded trajectory leaves the
// bounds of states 1..12 anywhere (sbnd: fill_bounds) -- checked on the fly,
// so the common case pays no separate pass (lazy_select runs only then).
template <int NS, bool WAVE = false>
__device__ __forceinline__ bool rti_expand(const RtiConst& C, int b, int l, const double w[NS], bool accept,
                                           const double* __restrict__ AB, const double* __restrict__ DEF,
                                           const double* __restrict__ Xb, const double* sbnd, double* vec,
                                           double* dxs) {
    const int N = C.N, n = C.n;
    // step safeguard (oracle rti_one): a failed QP (residual >= 1e-6 or NaN)
    // contributes no step; the shifted plan is kept and the gaps are closed
    if constexpr (WAVE) wave_sync(); else __syncthreads();
    {
        // column scale by value selects (a lane-dependent index into the
        // kernel-argument struct would copy it to scratch)
        const double iS0 = 1.0 / C.Su[0], iS1 = 1.0 / C.Su[1], iS2 = 1.0 / C.Su[2], iS3 = 1.0 / C.Su[3];
        const double iX13 = 1.0 / C.Sx13, iX14 = 1.0 / C.Sx14;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int i = l + 64 * s;
            const int c = i % 3;
            const double sc = i < 3 * N ? (c == 0 ? iS0 : (c == 1 ? iS1 : iS2))
                                        : (i < 4 * N ? iS3 : (i == 4 * N ? iX13 : iX14));
            if (i < n) vec[i] = accept ? w[s] * sc : 0.0;
        }
    }
    if constexpr (WAVE) wave_sync(); else __syncthreads();
    const double dth0 = vec[4 * N], dthd0 = vec[4 * N + 1];
    // theta / thetadot rows (exact double integrator), lane = node
    for (int k = l; k <= N; k += 64) {
        double dth = dth0 + (double)k * C.dt * dthd0, dthd = dthd0;
        for (int m = 0; m < k; ++m) {
            const double du = vec[3 * N + m];
            dth += C.dt * C.dt * ((double)(k - m) - 0.5) * du;
            dthd += C.dt * du;
        }
        dxs[k * 16 + 13] = dth;
        dxs[k * 16 + 14] = dthd;
    }
    // kite states: lane = row.  The recursion is a chain of N dependent steps:
    // dx_k is broadcast from lanes 0..12 by v_readlane (no LDS round trip), the
    // row dot product runs as four partial sums, and row l of [A_k | B_k] and
    // d_k come from a register ring PD intervals ahead (one interval of
    // look-ahead would expose a global-memory latency per interval).
    bool viol = false;
    {
        constexpr int PD = 4;
        double dx = 0.0;
        const double* ABb = AB + (size_t)b * N * NK * 16;
        const double* DEFb = DEF + (size_t)b * N * NK;
        const int lr = l < NK ? l : NK - 1;
        const double blo = sbnd[lr], bhi = sbnd[16 + lr];
        const double tlo = blo - bound_tol(blo), thi = bhi + bound_tol(bhi);
        const bool chk = l >= 1 && l < NK;             // states 1..12 (vx: a QP row)
        double ar[PD][16], dk[PD], xr[PD];
        auto fetch = [&](int k, double* a, double& d, double& xn) __attribute__((always_inline)) {
            const double* p = ABb + ((size_t)k * NK + lr) * 16;
#pragma unroll
            for (int j = 0; j < 16; ++j) a[j] = p[j];
            d = DEFb[(size_t)k * NK + lr];
            xn = Xb[(k + 1) * NX + lr];
        };
        auto interval = [&](int k, double* ring, double& dring, double& xring) __attribute__((always_inline)) {
            double a[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) a[j] = ring[j];
            const double d = dring, xn = xring;
            if (k + PD < N) fetch(k + PD, ring, dring, xring);
            double t0 = fma(a[NK], vec[3 * k], d), t1 = a[NK + 1] * vec[3 * k + 1];
            double t2 = a[NK + 2] * vec[3 * k + 2], t3 = 0.0;
#pragma unroll
            for (int j = 0; j < NK; j += 4) {
                t0 = fma(a[j], readlane_d(dx, j), t0);
                if (j + 1 < NK) t1 = fma(a[j + 1], readlane_d(dx, j + 1), t1);
                if (j + 2 < NK) t2 = fma(a[j + 2], readlane_d(dx, j + 2), t2);
                if (j + 3 < NK) t3 = fma(a[j + 3], readlane_d(dx, j + 3), t3);
            }
            dx = (t0 + t1) + (t2 + t3);
            if (l < NK) dxs[(k + 1) * 16 + l] = dx;
            const double xt = xn + dx;
            viol |= chk && (xt < tlo || xt > thi);
        };
        if (l < NK) dxs[l] = 0.0;
#pragma unroll
        for (int q = 0; q < PD; ++q)
            if (q < N) fetch(q, ar[q], dk[q], xr[q]);
        for (int k0 = 0; k0 < N; k0 += PD) {
            interval(k0, ar[0], dk[0], xr[0]);
            if (k0 + 1 >= N) break;
            interval(k0 + 1, ar[1], dk[1], xr[1]);
            if (k0 + 2 >= N) break;
            interval(k0 + 2, ar[2], dk[2], xr[2]);
            if (k0 + 3 >= N) break;
            interval(k0 + 3, ar[3], dk[3], xr[3]);
        }
    }
    if constexpr (WAVE) wave_sync(); else __syncthreads();
    return wave_or(viol ? 1 : 0) != 0;
}


template <bool WAVE = false>
__device__ __forceinline__ void rti_commit(const RtiConst& C, int b, int l, double kkt, int iters,
                                           const double* vec, const double* dxs, const double* sbnd,
                                           double* __restrict__ Xb, double* __restrict__ Ub,
                                           double* __restrict__ u0_out, double* __restrict__ diag,
                                           int32_t* __restrict__ status, double* __restrict__ kkt_out,
                                           int32_t* __restrict__ iters_out, int32_t* __restrict__ iters_acc,
                                           int B) {
    const int N = C.N;
    const bool accept = kkt < QP_STEP_ACCEPT;
    for (int k = l; k <= N; k += 64) {
        Xb[k * NX + 13] += dxs[k * 16 + 13];
        Xb[k * NX + 14] += dxs[k * 16 + 14];
    }
    for (int e = l; e < N * NU; e += 64) {
        const int k = e / NU, c = e % NU;
        Ub[e] += (c < 3) ? vec[3 * k + c] : vec[3 * N + k];
    }
    for (int e = l; e < N * NK; e += 64) {
        const int k = e / NK, i = e % NK;
        Xb[(k + 1) * NX + i] += dxs[(k + 1) * 16 + i];
    }
    if constexpr (WAVE) wave_sync(); else __syncthreads();

    // ---- diagnostics, cost, status -------------------------------------------
    double cost = 0.0, nrow = 0.0;
    int bad = 0, bound = 0;
    for (int k = l; k <= N; k += 64) {
        const double* xk = Xb + k * NX;
        double Pp[3], dP[3];
        path_eval(C, xk[13], Pp, dP);
        const bool last = (k == N);
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const double r = (last ? C.sqQ_T[a] : C.sqQ_dt[a]) * C.Sr[a] * (Pp[a] - xk[6 + a]);
            cost += r * r;
        }
        if (!last) {
            const double rv = C.sw * (C.sv * C.vref - C.sv * xk[14]);
            cost += rv * rv;
            for (int c = 0; c < NU; ++c) {
                const double su = C.Su[c] * Ub[k * NU + c];
                cost += C.dt * C.Rraw[c] * su * su;
            }
        }
        for (int i = 0; i < NX; ++i) if (!isfinite(xk[i])) bad = 1;
        if (k < N) for (int c = 0; c < NU; ++c) if (!isfinite(Ub[k * NU + c])) bad = 1;
        if (k >= 1)
            for (int i = 1; i < 13; ++i) {
                const double lb = sbnd[i], ub = sbnd[16 + i];
                if (xk[i] < lb - bound_tol(lb) || xk[i] > ub + bound_tol(ub)) { bound = 1; nrow += 1.0; }
            }
    }
    cost = wave_sum(cost);
    nrow = wave_sum(nrow);
    bad = wave_or(bad);
    bound = wave_or(bound);
    if (l == 0) {
        double Pp[3], dP[3];
        path_eval(C, Xb[13], Pp, dP);
        double pe = 0.0;
        for (int a = 0; a < 3; ++a) { const double e = C.Sr[a] * (Pp[a] - Xb[6 + a]); pe += e * e; }
        double* dg = diag + (size_t)b * 6;
        dg[0] = sqrt(pe);
        dg[1] = fabs(C.sv * C.vref - C.sv * Xb[14]);
        dg[2] = cost;
        dg[3] = Xb[13];
        dg[4] = Ub[3];
        dg[5] = kkt;
        int32_t st = status[b];
        if (bad) st |= 1;
        if (!(kkt < 1e-8)) st |= 2;
        if (!accept) st |= 32;
        if (bound && !bad) st |= 8;
        status[b] = st;
        if (kkt_out) kkt_out[b] = kkt;
        if (iters_out) iters_out[b] = iters;
        if (iters_acc) {                               // running sums since kite_nmpc_timing_start
            iters_acc[b] += iters;
            iters_acc[B + b] += (bound && !bad) ? 1 : 0;        // kite-steps ending outside the state box
            iters_acc[2 * B + b] += bad ? 0 : (int32_t)nrow;    // (node, state) pairs outside it
        }
        for (int c = 0; c < NU; ++c) u0_out[(size_t)b * NU + c] = Ub[c];
    }
}

// ---- lazy state-bound rows (oracle rti_one, LAZY_ROWS / LAZY_ROUNDS) --------
// The vx bound is a QP row at every node; the other finite state bounds are
// enforced on demand: after an accepted QP solve the expanded trajectory is
// checked (states 1..12, nodes 1..N), the most violated (node, state) pairs
// -- largest normalised violation first, ties by node then state, at most
// LAZY_ROWS per RTI step -- become QP rows +-G_k[i,:] D w >= c, and the QP is
// solved again from a cold start, at most LAZY_ROUNDS times.
constexpr int LAZY_ROWS = 4, LAZY_ROUNDS = 2;
constexpr int QP_LAZY_GRID = 256;                  // blocks of the lazy instances (grid-stride)
// Every QP kernel comes in two instances.  LAZY = false (the whole grid)
// solves, expands and checks the state bounds on the fly (rti_expand); a kite
// with violations is appended to a list (lazy[0] = count, lazy[1..] = kites;
// count reset by k_qp_order) and left uncommitted.  LAZY = true (launched
// next, a 256-block grid-stride loop over the list) runs the full rule -- the
// identical first solve, then the rounds with rows -- for the listed kites.
// The fast instance thus has no re-solve loop (the back edge alone costs the
// tiled kernel ~350 B/lane of spills) and the lazy one costs ~2 us when the
// list is empty.
// bound table (LDS): sbnd[i] = lbx[i], sbnd[16 + i] = ubx[i]
__device__ __forceinline__ void fill_bounds(const RtiConst& C, int l, double* sbnd) {
#pragma unroll
    for (int i = 0; i < NX; ++i)
        if (l == i) { sbnd[i] = C.lbx[i]; sbnd[16 + i] = C.ubx[i]; }
}
// Violations of the trajectory Xb + dxs -> viol[(k-1)*12 + (i-1)] (signed
// normalised magnitude: > 0 below lb, < 0 above ub), then the `want` largest
// into sel[3t + {0,1,2}] = {k, i, side}; returns their count (wave-uniform).
template <bool WAVE = false>
__device__ __attribute__((noinline)) int lazy_select(const RtiConst& C, int l, const double* Xb, const double* dxs, const double* sbnd,
                           double* viol, int* sel, int want) {
    const int N = C.N, np = N * 12;
    for (int p = l; p < np; p += 64) {
        const int k = 1 + p / 12, i = 1 + p % 12;
        const double lb = sbnd[i], ub = sbnd[16 + i];
        const double x = Xb[k * NX + i] + dxs[k * 16 + i];
        double v = 0.0;
        if (x < lb - bound_tol(lb)) v = (lb - x) / fmax(1.0, fabs(lb));
        else if (x > ub + bound_tol(ub)) v = -(x - ub) / fmax(1.0, fabs(ub));
        viol[p] = v;
    }
    if constexpr (WAVE) wave_sync(); else __syncthreads();
    int cnt = 0;
    for (int t = 0; t < want; ++t) {
        double best = 0.0, bp = 1e9;
        for (int p = l; p < np; p += 64) {
            const double a = fabs(viol[p]);
            if (a > best) { best = a; bp = (double)p; }
        }
        const double M = wave_max(best);
        if (!(M > 0.0)) break;
        const int pm = (int)wave_min(best == M ? bp : 1e9);
        if constexpr (WAVE) wave_sync(); else __syncthreads();
        if (l == 0) {
            sel[3 * t] = 1 + pm / 12;
            sel[3 * t + 1] = 1 + pm % 12;
            sel[3 * t + 2] = viol[pm] > 0.0 ? 1 : -1;
            viol[pm] = 0.0;
        }
        if constexpr (WAVE) wave_sync(); else __syncthreads();
        ++cnt;
    }
    return cnt;
}
// QP row of the violated (node k, state i, side): row[3j + c] = side G_k[i, (j, c)] / Su_c
// for the kite controls (zero from column 3k on; theta and Uv columns are zero
// for kite states), by the backward recursion lambda_j = A_j' lambda_{j+1},
// lambda_k = e_i; returns the bound c of  row . w >= c  (wsc: scaled w, LDS).
// row[0, ncol) is written (ncol >= 3N: the caller's row stride).
template <bool WAVE = false>
__device__ double lazy_row(const RtiConst& C, int b, int l, int k, int i, int side, const double* __restrict__ AB,
                           const double* Xb, const double* dxs, const double* sbnd, const double* wsc,
                           double* row, int ncol) {
    const int N = C.N;
    const double iS0 = 1.0 / C.Su[0], iS1 = 1.0 / C.Su[1], iS2 = 1.0 / C.Su[2];
    for (int j = l; j < ncol; j += 64) row[j] = 0.0;
    if constexpr (WAVE) wave_sync(); else __syncthreads();
    double lam = (l == i) ? (double)side : 0.0;
    const double* ABb = AB + (size_t)b * N * NK * 16;
    for (int j = k - 1; j >= 0; --j) {
        const double* a = ABb + (size_t)j * NK * 16 + (l & 15);
        double acc = 0.0;
#pragma unroll
        for (int r = 0; r < NK; ++r) acc = fma(readlane_d(lam, r), a[r * 16], acc);
        if (l >= NK && l < 16) {
            const int c = l - NK;
            row[3 * j + c] = acc * (c == 0 ? iS0 : (c == 1 ? iS1 : iS2));
        }
        lam = l < NK ? acc : 0.0;
    }
    if constexpr (WAVE) wave_sync(); else __syncthreads();
    const double bnd = side > 0 ? sbnd[i] : sbnd[16 + i];
    const double xtry = Xb[k * NX + i] + dxs[k * 16 + i];
    double dot = 0.0;
    for (int j = l; j < 3 * k; j += 64) dot = fma(row[j], wsc[j], dot);
    return (double)side * (bnd - xtry) + wave_sum(dot);
}

// start point s = max(g, 0.1), z = 20 (oracle qp_ipm; z0 = 20 cuts the N = 20
// closed loop's mean IPM iterations from 11.68 to 11.11 against z0 = 10,
// profiles/r04_oracle_n20_z0_study.txt)
constexpr double IPM_S0 = 0.1, IPM_Z0 = 20.0, IPM_FREEZE = 1e-10, IPM_TAU = 0.995;
// stalled IPM (oracle IPM_MU_FLOOR): complementarity exhausted (mu < 1e-20)
// while a rounding floor of the stationarity residual keeps the test above the
// freeze; continuing drives s, z to underflow and the Newton system to NaN
constexpr double IPM_MU_FLOOR = 1e-20;
// k_qp_tiled's recursive residuals (oracle cfg C_qp_rec, qp_tiled.inc)
constexpr double QP_REC_THR = 1e-6;
__device__ __forceinline__ int pk(int i, int c) { return (i * (i + 1)) / 2 + c; }

// row of element e in a row-wise packed lower triangle
__device__ __forceinline__ int tri_row(int e) {
    int r = (int)((sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);
    if ((r + 1) * (r + 2) / 2 <= e) ++r;
    if (r * (r + 1) / 2 > e) --r;
    return r;
}

// variable k of a slot vector (i = l + 64 s), broadcast to the wave
template <int NS>
__device__ __forceinline__ double slot_pivot(double x[NS], int k, int l) {
    double v = x[0];
#pragma unroll
    for (int s = 1; s < NS; ++s) v = (k >= 64 * s) ? x[s] : v;
    return readlane_d(v, k & 63);
}

template <int NS>
struct QPState {
    // per-lane slots: variable i = l + 64*s (s = 0 .. NS-1)
    double w[NS], lb[NS], ub[NS], h[NS], sl[NS], zl[NS], su[NS], zu[NS];
    double rd[NS], rpl[NS], rpu[NS];
    // general rows: lane k < N
    double clo, chi, slo, zlo, shi, zhi, rplo, rphi, cw;
};

// NQ: largest n = 4N + 2 of the instantiation (82: N <= 20, 162: N <= 40);
// C (vx-bound rows) is stored on its 3N kite columns only.
template <int NQ, bool LAZY>
__device__ __forceinline__ void qp_body(int b, ModelConst /*P*/, RtiConst C, int B,
                                           const double* __restrict__ Hs, const double* __restrict__ hs,
                                           const double* __restrict__ Cr, const double* __restrict__ clp,
                                           const double* __restrict__ cup, const double* __restrict__ hmaxp,
                                           const double* __restrict__ AB, const double* __restrict__ DEF,
                                           double* __restrict__ X, double* __restrict__ U,
                                           double* __restrict__ u0_out, double* __restrict__ diag,
                                           int32_t* __restrict__ status, double* __restrict__ kkt_out,
                                           int32_t* __restrict__ iters_out, int32_t* __restrict__ lazy) {
    constexpr int NS = (NQ + 63) / 64;                 // variable slots per lane
    constexpr int NQN = (NQ - 2) / 4;                  // largest horizon
    __shared__ double Lp[NQ * (NQ + 1) / 2];
    __shared__ double sC[(NQN + LAZY_ROWS) * 3 * NQN];   // vx rows, then the lazy state-bound rows
    __shared__ double vec[NQ + 2];
    __shared__ double col[NQ];
    __shared__ double dinv[NQ];
    __shared__ double eq[NQ];          // equilibration E = diag(M)^-1/2 of the current factorization
    __shared__ double sbnd[32], sXc[LAZY_ROWS];
    __shared__ int sel[3 * LAZY_ROWS];

    const int l = threadIdx.x;
    const int N = C.N, n = C.n;
    const double* Hb = Hs + (size_t)b * n * n;
    const double* Crb = Cr + (size_t)b * N * n;
    double* Xb = X + (size_t)b * (N + 1) * NX;
    double* Ub = U + (size_t)b * N * NU;

    const int nc = 3 * N;                             // C columns kept (kite controls)
    for (int e = l; e < N * nc; e += 64) sC[e] = Crb[(e / nc) * n + e % nc];
    fill_bounds(C, l, sbnd);

    QPState<NS> q;
    const bool has_lo = C.lo_fin != 0, has_hi = C.hi_fin != 0;
    int m = N;                                        // rows in use: N vx rows + lazy rows
    int nI = 2 * n + N * ((has_lo ? 1 : 0) + (has_hi ? 1 : 0));
    bool row_lane = l < N;
    bool rlo = row_lane && has_lo, rhi = row_lane && has_hi;   // this row lane's finite sides
    auto init_ipm = [&]() {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const int i = l + 64 * s;
        double lo = 0.0, hi = 0.0, hv = 0.0;
        if (i < n) {
            if (i < 3 * N) {
                const int k = i / 3, c = i % 3;
                lo = C.Su[c] * (C.lbu[c] - Ub[k * NU + c]);
                hi = C.Su[c] * (C.ubu[c] - Ub[k * NU + c]);
            } else if (i < 4 * N) {
                const int k = i - 3 * N;
                lo = C.Su[3] * (C.lbu[3] - Ub[k * NU + 3]);
                hi = C.Su[3] * (C.ubu[3] - Ub[k * NU + 3]);
            } else if (i == 4 * N) {
                lo = -C.flex * C.Sx13; hi = C.flex * C.Sx13;
            } else {
                lo = -C.flex * C.Sx14; hi = C.flex * C.Sx14;
            }
            hv = hs[(size_t)b * n + i];
        }
        q.lb[s] = lo; q.ub[s] = hi; q.h[s] = hv;
        const double mar = 0.1 * (hi - lo);
        double w0 = 0.0;
        if (w0 < lo + mar) w0 = lo + mar;
        if (w0 > hi - mar) w0 = hi - mar;
        q.w[s] = (i < n) ? w0 : 0.0;
        q.sl[s] = fmax(q.w[s] - lo, IPM_S0);
        q.su[s] = fmax(hi - q.w[s], IPM_S0);
        q.zl[s] = IPM_Z0; q.zu[s] = IPM_Z0;
    }
    q.clo = l < N ? clp[(size_t)b * N + l] : (row_lane ? sXc[l - N] : 0.0);
    q.chi = l < N ? cup[(size_t)b * N + l] : 0.0;
    };
    init_ipm();
    const double dscale = 1.0 / (1.0 + hmaxp[b]);

    // --- helpers ---------------------------------------------------------
    // y = C x for row lanes, x given in vec[]
    auto rows_times = [&]() -> double {
        double t = 0.0;
        if (row_lane) {
            const double* cr = sC + l * nc;
            for (int j = 0; j < nc; ++j) t = fma(cr[j], vec[j], t);
        }
        return t;
    };
    // out_s = C^T y (y given in vec[] for rows)
    auto rows_T = [&](double out[NS]) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int i = l + 64 * s;
            double t = 0.0;
            if (i < n)
                if (i < nc)
                    for (int k = 0; k < m; ++k) t = fma(sC[k * nc + i], vec[k], t);
            out[s] = t;
        }
    };
    auto put_vec2 = [&](const double a[NS]) {
#pragma unroll
        for (int s = 0; s < NS; ++s) { const int i = l + 64 * s; if (i < n) vec[i] = a[s]; }
    };

    // initial slacks of general rows
    auto init_rows = [&]() {
        put_vec2(q.w);
        __syncthreads();
        q.cw = rows_times();
        q.slo = rlo ? fmax(q.cw - q.clo, IPM_S0) : 1.0;
        q.shi = rhi ? fmax(q.chi - q.cw, IPM_S0) : 1.0;
        q.zlo = rlo ? IPM_Z0 : 0.0;
        q.zhi = rhi ? IPM_Z0 : 0.0;
        __syncthreads();
    };
    init_rows();

    double resid = 0.0;
    auto residuals = [&]() -> double {
        // vec <- w ; Hw (column sweep, H symmetric), Cw
        put_vec2(q.w);
        __syncthreads();
        double hw[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) hw[s] = 0.0;
        for (int j = 0; j < n; ++j) {
            const double wj = vec[j];
            const double* hr = Hb + (size_t)j * n;
#pragma unroll
            for (int s = 0; s < NS; ++s)
                if (l + 64 * s < n) hw[s] = fma(hr[l + 64 * s], wj, hw[s]);
        }
        q.cw = rows_times();
        __syncthreads();
        if (row_lane) vec[l] = (rlo ? q.zlo : 0.0) - (rhi ? q.zhi : 0.0);
        __syncthreads();
        double ctz[NS];
        rows_T(ctz);
        __syncthreads();
        double rmax = 0.0, mu = 0.0;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int i = l + 64 * s;
            if (i < n) {
                q.rd[s] = hw[s] + q.h[s] - (q.zl[s] - q.zu[s]) - ctz[s];
                q.rpl[s] = q.w[s] - q.lb[s] - q.sl[s];
                q.rpu[s] = q.ub[s] - q.w[s] - q.su[s];
                rmax = nmax(rmax, fabs(q.rd[s]) * dscale);
                rmax = nmax(rmax, fmax(fabs(q.rpl[s]), fabs(q.rpu[s])));
                mu += q.sl[s] * q.zl[s] + q.su[s] * q.zu[s];
            } else {
                q.rd[s] = 0.0; q.rpl[s] = 0.0; q.rpu[s] = 0.0;
            }
        }
        q.rplo = 0.0; q.rphi = 0.0;
        if (rlo) { q.rplo = q.cw - q.clo - q.slo; rmax = nmax(rmax, fabs(q.rplo)); mu += q.slo * q.zlo; }
        if (rhi) { q.rphi = q.chi - q.cw - q.shi; rmax = nmax(rmax, fabs(q.rphi)); mu += q.shi * q.zhi; }
        rmax = wave_nmax(rmax);
        mu = wave_sum(mu) / (double)nI;
        resid = nmax(rmax, mu);
        return mu;
    };

    // Cholesky of the packed matrix in Lp (in place, lower)
    auto cholesky = [&]() {
        for (int j = 0; j < n; ++j) {
            const double piv = piv_fix(Lp[pk(j, j)]);
            const double dj = sqrt(piv);
            const double inv = 1.0 / dj;
            __syncthreads();
            if (l == 0) { Lp[pk(j, j)] = dj; dinv[j] = inv; }
            for (int i = j + 1 + l; i < n; i += 64) {
                const double vv = Lp[pk(i, j)] * inv;
                Lp[pk(i, j)] = vv;
                col[i - j - 1] = vv;
            }
            __syncthreads();
            const int m = n - j - 1;
            const int T = m * (m + 1) / 2;
            for (int e = l; e < T; e += 64) {
                const int ip = tri_row(e);
                const int cp = e - ip * (ip + 1) / 2;
                const int idx = pk(j + 1 + ip, j + 1 + cp);
                Lp[idx] = fma(-col[ip], col[cp], Lp[idx]);
            }
            __syncthreads();
        }
    };
    // x <- M^-1 x = E (E M E)^-1 E x with x in per-lane slots (NS); Lp holds
    // the factor of E M E
    auto chol_solve = [&](double x[NS]) {
#pragma unroll
        for (int s = 0; s < NS; ++s) { const int i = l + 64 * s; if (i < n) x[s] *= eq[i]; }
        for (int k = 0; k < n; ++k) {
            double xk;
            xk = slot_pivot<NS>(x, k, l) * dinv[k];
#pragma unroll
            for (int s = 0; s < NS; ++s)
                if (l + 64 * s == k) x[s] = xk;
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const int i = l + 64 * s;
                if (i > k && i < n) x[s] = fma(-Lp[pk(i, k)], xk, x[s]);
            }
        }
        for (int k = n - 1; k >= 0; --k) {
            double xk;
            xk = slot_pivot<NS>(x, k, l) * dinv[k];
#pragma unroll
            for (int s = 0; s < NS; ++s)
                if (l + 64 * s == k) x[s] = xk;
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const int i = l + 64 * s;
                if (i < k) x[s] = fma(-Lp[pk(k, i)], xk, x[s]);
            }
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) { const int i = l + 64 * s; if (i < n) x[s] *= eq[i]; }
    };

    double sgl[NS], sgu[NS], sglo = 0.0, sghi = 0.0;
    // Newton solve for complementarity rhs rc; returns directions
    struct Dir { double dw[NS], dsl[NS], dsu[NS], dzl[NS], dzu[NS], dslo, dshi, dzlo, dzhi; };
    auto newton = [&](const double rcl[NS], const double rcu[NS], double rclo, double rchi, Dir& D) {
        double t_lo = 0.0, t_hi = 0.0;
        if (rlo) t_lo = rclo / q.slo - sglo * q.rplo;
        if (rhi) t_hi = rchi / q.shi - sghi * q.rphi;
        __syncthreads();
        if (row_lane) vec[l] = t_lo - t_hi;
        __syncthreads();
        double ct[NS];
        rows_T(ct);
        double r[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int i = l + 64 * s;
            if (i < n) {
                const double tl = rcl[s] / q.sl[s] - sgl[s] * q.rpl[s];
                const double tu = rcu[s] / q.su[s] - sgu[s] * q.rpu[s];
                r[s] = -q.rd[s] + (tl - tu) + ct[s];
            } else {
                r[s] = 0.0;
            }
        }
        chol_solve(r);
        __syncthreads();
        put_vec2(r);
        __syncthreads();
        const double cdw = rows_times();
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            D.dw[s] = r[s];
            D.dsl[s] = r[s] + q.rpl[s];
            D.dsu[s] = -r[s] + q.rpu[s];
            D.dzl[s] = (rcl[s] - q.zl[s] * D.dsl[s]) / q.sl[s];
            D.dzu[s] = (rcu[s] - q.zu[s] * D.dsu[s]) / q.su[s];
        }
        D.dslo = 0.0; D.dshi = 0.0; D.dzlo = 0.0; D.dzhi = 0.0;
        if (rlo) { D.dslo = cdw + q.rplo; D.dzlo = (rclo - q.zlo * D.dslo) / q.slo; }
        if (rhi) { D.dshi = -cdw + q.rphi; D.dzhi = (rchi - q.zhi * D.dshi) / q.shi; }
    };
    auto max_step = [&](const Dir& D) -> double {
        double a = 1.0;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int i = l + 64 * s;
            if (i < n) {
                if (D.dsl[s] < 0.0) a = fmin(a, -q.sl[s] / D.dsl[s]);
                if (D.dsu[s] < 0.0) a = fmin(a, -q.su[s] / D.dsu[s]);
                if (D.dzl[s] < 0.0) a = fmin(a, -q.zl[s] / D.dzl[s]);
                if (D.dzu[s] < 0.0) a = fmin(a, -q.zu[s] / D.dzu[s]);
            }
        }
        if (rlo) {
            if (D.dslo < 0.0) a = fmin(a, -q.slo / D.dslo);
            if (D.dzlo < 0.0) a = fmin(a, -q.zlo / D.dzlo);
        }
        if (rhi) {
            if (D.dshi < 0.0) a = fmin(a, -q.shi / D.dshi);
            if (D.dzhi < 0.0) a = fmin(a, -q.zhi / D.dzhi);
        }
        return wave_min(a);
    };

    int iters = C.K;
    double kkt = 0.0;
    double* dxs = Lp;                                 // the factor is dead after the last solve
    double* viol = Lp + (N + 1) * 16;
    for (int round = 0, added = 0;; ++round) {
    iters = C.K;
    for (int it = 0; it < C.K; ++it) {
        const double mu = residuals();
        if (resid < IPM_FREEZE || resid != resid || mu < IPM_MU_FLOOR) { iters = it; break; }   // converged, poisoned or stalled
        // sigma = z/s and the normal matrix H + A' Sigma A into Lp
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            sgl[s] = q.zl[s] / q.sl[s];
            sgu[s] = q.zu[s] / q.su[s];
        }
        sglo = rlo ? q.zlo / q.slo : 0.0;
        sghi = rhi ? q.zhi / q.shi : 0.0;
        __syncthreads();
        if (row_lane) vec[l] = sglo + sghi;
        __syncthreads();
        for (int rr = 0; rr < n; ++rr) {
            const double* hr = Hb + (size_t)rr * n;
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const int c = l + 64 * s;
                if (c <= rr) {
                    double mv = hr[c];
                    if (rr < nc && c < nc)
                        for (int k = 0; k < m; ++k) mv = fma(sC[k * nc + rr] * vec[k], sC[k * nc + c], mv);
                    if (c == rr) mv += sgl[s] + sgu[s];
                    Lp[pk(rr, c)] = mv;
                }
            }
        }
        __syncthreads();
        // equilibrate M <- E M E, E = diag(M)^-1/2 (as k_qp_tiled / k_qp_lds):
        // near convergence the barrier weights spread the diagonal over ~24
        // decades, and unequilibrated the last factorizations of an ill-
        // conditioned QP (N = 40: a pivot at 4e-15 of its diagonal) left the
        // step along the Hessian's near-null directions to rounding
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int i = l + 64 * s;
            if (i < n) eq[i] = 1.0 / sqrt(piv_fix(Lp[pk(i, i)]));
        }
        __syncthreads();
        for (int rr = 0; rr < n; ++rr) {
            const double er = eq[rr];
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const int c = l + 64 * s;
                if (c <= rr) Lp[pk(rr, c)] *= er * eq[c];
            }
        }
        __syncthreads();
        cholesky();
        // predictor
        double rcl[NS], rcu[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) { rcl[s] = -q.sl[s] * q.zl[s]; rcu[s] = -q.su[s] * q.zu[s]; }
        double rclo = -q.slo * q.zlo, rchi = -q.shi * q.zhi;
        Dir Da;
        newton(rcl, rcu, rclo, rchi, Da);
        const double aa = max_step(Da);
        double mua = 0.0;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int i = l + 64 * s;
            if (i < n)
                mua += (q.sl[s] + aa * Da.dsl[s]) * (q.zl[s] + aa * Da.dzl[s]) +
                       (q.su[s] + aa * Da.dsu[s]) * (q.zu[s] + aa * Da.dzu[s]);
        }
        if (rlo) mua += (q.slo + aa * Da.dslo) * (q.zlo + aa * Da.dzlo);
        if (rhi) mua += (q.shi + aa * Da.dshi) * (q.zhi + aa * Da.dzhi);
        mua = wave_sum(mua) / (double)nI;
        double sigma = mua / mu;
        sigma = sigma * sigma * sigma;
        // corrector
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            rcl[s] = -q.sl[s] * q.zl[s] - Da.dsl[s] * Da.dzl[s] + sigma * mu;
            rcu[s] = -q.su[s] * q.zu[s] - Da.dsu[s] * Da.dzu[s] + sigma * mu;
        }
        rclo = rlo ? -q.slo * q.zlo - Da.dslo * Da.dzlo + sigma * mu : 0.0;
        rchi = rhi ? -q.shi * q.zhi - Da.dshi * Da.dzhi + sigma * mu : 0.0;
        Dir Dc;
        newton(rcl, rcu, rclo, rchi, Dc);
        const double a = fmin(1.0, fmax(IPM_TAU, 1.0 - mu) * max_step(Dc));   // tau_k -> 1 (oracle qp_ipm)
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            q.w[s] += a * Dc.dw[s];
            q.sl[s] += a * Dc.dsl[s]; q.su[s] += a * Dc.dsu[s];
            q.zl[s] += a * Dc.dzl[s]; q.zu[s] += a * Dc.dzu[s];
        }
        if (rlo) { q.slo += a * Dc.dslo; q.zlo += a * Dc.dzlo; }
        if (rhi) { q.shi += a * Dc.dshi; q.zhi += a * Dc.dzhi; }
    }
    // final residual (also when frozen: residuals() already ran)
    residuals();
    kkt = resid;
    __syncthreads();
    const bool outside = rti_expand<NS>(C, b, l, q.w, kkt < QP_STEP_ACCEPT, AB, DEF, Xb, sbnd, vec, dxs);
    if (!outside || !(kkt < QP_STEP_ACCEPT) || round == LAZY_ROUNDS || added == LAZY_ROWS) break;
    const int cnt = lazy_select(C, l, Xb, dxs, sbnd, viol, sel, LAZY_ROWS - added);
    if (cnt == 0) break;
    if constexpr (!LAZY) { if (l == 0) lazy[1 + atomicAdd(lazy, 1)] = b; return; }   // to the lazy instance
#pragma unroll
    for (int s = 0; s < NS; ++s) { const int i = l + 64 * s; if (i < n) col[i] = q.w[s]; }   // scaled w
    __syncthreads();
    for (int t = 0; t < cnt; ++t) {
        const double cv = lazy_row(C, b, l, sel[3 * t], sel[3 * t + 1], sel[3 * t + 2], AB, Xb, dxs, sbnd, col,
                                   sC + (size_t)m * nc, nc);
        if (l == 0) sXc[m - N] = cv;
        ++m;
        __syncthreads();
    }
    added += cnt;
    // the QP again with the new rows (cold start)
    nI += cnt;
    row_lane = l < m;
    rlo = l < N ? (row_lane && has_lo) : row_lane;
    rhi = l < N ? (row_lane && has_hi) : false;
    init_ipm();
    init_rows();
    }
    rti_commit(C, b, l, kkt, iters, vec, dxs, sbnd, Xb, Ub, u0_out, diag, status, kkt_out, iters_out,
               iters_out ? iters_out + B : nullptr, B);
}

// the fast instance over the whole grid (LPT order); the lazy instance over
// the kites the fast one listed (lazy[0] = count, lazy[1..]), grid-strided
// (separate names: profilers that truncate template arguments keep them apart)
template <int NQ>
__global__ __launch_bounds__(64) void k_qp(ModelConst P, RtiConst C, int B,
                                           const double* __restrict__ Hs, const double* __restrict__ hs,
                                           const double* __restrict__ Cr, const double* __restrict__ clp,
                                           const double* __restrict__ cup, const double* __restrict__ hmaxp,
                                           const double* __restrict__ AB, const double* __restrict__ DEF,
                                           double* __restrict__ X, double* __restrict__ U,
                                           double* __restrict__ u0_out, double* __restrict__ diag,
                                           int32_t* __restrict__ status, double* __restrict__ kkt_out,
                                           int32_t* __restrict__ iters_out,
                                           const int32_t* __restrict__ order, int32_t* __restrict__ lazy) {
        qp_body<NQ, false>(order ? order[blockIdx.x] : blockIdx.x, P, C, B, Hs, hs, Cr, clp, cup, hmaxp, AB, DEF, X, U, u0_out, diag, status, kkt_out, iters_out, lazy);
}
template <int NQ>
__global__ __launch_bounds__(64) void k_qp_lazy(ModelConst P, RtiConst C, int B,
                                           const double* __restrict__ Hs, const double* __restrict__ hs,
                                           const double* __restrict__ Cr, const double* __restrict__ clp,
                                           const double* __restrict__ cup, const double* __restrict__ hmaxp,
                                           const double* __restrict__ AB, const double* __restrict__ DEF,
                                           double* __restrict__ X, double* __restrict__ U,
                                           double* __restrict__ u0_out, double* __restrict__ diag,
                                           int32_t* __restrict__ status, double* __restrict__ kkt_out,
                                           int32_t* __restrict__ iters_out,
                                           const int32_t* __restrict__ order, int32_t* __restrict__ lazy) {
        const int cnt = lazy[0];
        for (int j = blockIdx.x; j < cnt; j += gridDim.x) {
            qp_body<NQ, true>(lazy[1 + j], P, C, B, Hs, hs, Cr, clp, cup, hmaxp, AB, DEF, X, U, u0_out, diag, status, kkt_out, iters_out, lazy);
            __syncthreads();
        }
}

// ---------------------------------------------------------------------------
// model-level utility kernels (lane per item)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64, 2) void k_dynamics(ModelConst P, int count, const double* __restrict__ x,
                           const double* __restrict__ u, double* __restrict__ f) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    double xx[NK], uu[NKU], ff[NK];
    for (int j = 0; j < NK; ++j) xx[j] = x[(size_t)i * NX + j];
    for (int j = 0; j < NKU; ++j) uu[j] = u[(size_t)i * NU + j];
    kite_rhs<double>(P, xx, uu, ff);
    for (int j = 0; j < NK; ++j) f[(size_t)i * NX + j] = ff[j];
    f[(size_t)i * NX + 13] = x[(size_t)i * NX + 14];
    f[(size_t)i * NX + 14] = u[(size_t)i * NU + 3];
}

// lane = (item, direction): 16 directions per item
__global__ __launch_bounds__(256, 2) void k_jacobian(ModelConst P, int count, const double* __restrict__ x,
                           const double* __restrict__ u, double* __restrict__ Jx,
                           double* __restrict__ Ju) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = g >> 4, d = g & 15;
    if (i >= count) return;
    Dual xx[NK], uu[NKU], ff[NK];
    for (int j = 0; j < NK; ++j) xx[j] = mk(x[(size_t)i * NK + j], d == j ? 1.0 : 0.0);
    for (int j = 0; j < NKU; ++j) uu[j] = mk(u[(size_t)i * NKU + j], d == NK + j ? 1.0 : 0.0);
    kite_rhs<Dual>(P, xx, uu, ff);
    for (int r = 0; r < NK; ++r) {
        if (d < NK) Jx[((size_t)i * NK + r) * NK + d] = ff[r].t;
        else Ju[((size_t)i * NK + r) * NKU + (d - NK)] = ff[r].t;
    }
}

__global__ __launch_bounds__(64, 2) void k_predict(ModelConst P, int count, const double* __restrict__ x,
                          const double* __restrict__ u, double h, int steps,
                          double* __restrict__ xo) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    double xx[NX], uu[NU], yy[NX];
    for (int j = 0; j < NX; ++j) xx[j] = x[(size_t)i * NX + j];
    for (int j = 0; j < NU; ++j) uu[j] = u[(size_t)i * NU + j];
    rk4_primal(P, xx, uu, h, steps, yy);
    for (int j = 0; j < NX; ++j) xo[(size_t)i * NX + j] = yy[j];
}

// rk4 with sensitivities for independent (x,u) items (API kite_nmpc_rk4_sens):
// the items run through the hot kernel k_rk4_sens2 itself as a batch of
// one-interval horizons (N = 1, node 1 = 0 so the "defect" is x+), then
// k_sens_items_expand writes the full 15x15 / 15x4 blocks with the exact
// theta/thetadot/Uv rows and columns.  X2 [count][2][15] is scratch.
__global__ __launch_bounds__(64) void k_sens_items_stage(int count, const double* __restrict__ x,
                                                         double* __restrict__ X2) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= count * 2 * NX) return;
    const int i = g / (2 * NX), e = g % (2 * NX);
    X2[g] = e < NX ? x[(size_t)i * NX + e] : 0.0;
}
// lane per (item, row r of [A | B]): 15 rows per item
__global__ __launch_bounds__(64) void k_sens_items_expand(int count, int M, double h, const double* __restrict__ x,
                                                          const double* __restrict__ u,
                                                          const double* __restrict__ AB,
                                                          const double* __restrict__ DEF, double* __restrict__ xo,
                                                          double* __restrict__ A, double* __restrict__ Bm) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= count * NX) return;
    const int i = g / NX, r = g % NX;
    const double T = h * M;
    double* Ar = A + ((size_t)i * NX + r) * NX;
    double* Br = Bm + ((size_t)i * NX + r) * NU;
    const double* xi = x + (size_t)i * NX;
    if (r < NK) {
        const double* ab = AB + ((size_t)i * NK + r) * 16;
        for (int c = 0; c < NK; ++c) Ar[c] = ab[c];
        Ar[13] = 0.0; Ar[14] = 0.0;
        for (int c = 0; c < NKU; ++c) Br[c] = ab[NK + c];
        Br[3] = 0.0;
        xo[(size_t)i * NX + r] = DEF[(size_t)i * NK + r];
    } else {
        for (int c = 0; c < NX; ++c) Ar[c] = 0.0;
        for (int c = 0; c < NU; ++c) Br[c] = 0.0;
        const double uv = u[(size_t)i * NU + 3];
        if (r == 13) {
            Ar[13] = 1.0; Ar[14] = T; Br[3] = 0.5 * T * T;
            xo[(size_t)i * NX + 13] = xi[13] + T * xi[14] + 0.5 * T * T * uv;
        } else {
            Ar[14] = 1.0; Br[3] = T;
            xo[(size_t)i * NX + 14] = xi[14] + T * uv;
        }
    }
}

// findClosestPointOnPath (kiteNMPF.cpp:358-391): gradient steps on
// 0.5*||P(theta) - pos|| with step 0.25, tol 1e-2, <= 11 updates.
__global__ __launch_bounds__(64, 2) void k_closest_point(RtiConst C, int count, const double* __restrict__ pos,
                                const double* __restrict__ guess, double* __restrict__ theta) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    theta[i] = closest_point_dev(C, pos[(size_t)i * 3], pos[(size_t)i * 3 + 1], pos[(size_t)i * 3 + 2],
                                 guess ? guess[i] : 0.0);
}

// ---------------------------------------------------------------------------
// launch wrappers
// ---------------------------------------------------------------------------
hipError_t launch_prologue(const ModelConst& P, const RtiConst& C, int B, int warm, const double* x0,
                           double* X, double* U, int32_t* status, const double* wind, int32_t* cold,
                           hipStream_t s) {
    constexpr int PRO_COLD_GRID = 256;
    if (warm && !(C.delay > 0.0)) {
        hipLaunchKernelGGL(k_prologue_warm, dim3(B), dim3(64), 0, s, P, C, B, x0, X, U, status, cold);
        hipLaunchKernelGGL(k_prologue_cold, dim3(B < PRO_COLD_GRID ? B : PRO_COLD_GRID), dim3(64), 0, s, P, C,
                           x0, X, U, status, wind, cold, B);
    } else {
        hipLaunchKernelGGL(k_prologue, dim3(B), dim3(64), 0, s, P, C, B, warm, x0, X, U, status, wind);
    }
    return hipGetLastError();
}
hipError_t launch_rk4_sens(const ModelConst& P, const RtiConst& C, int B, const double* X, const double* U,
                           double* AB, double* DEF, const double* wind, hipStream_t s) {
    const dim3 grid2((B + RK2_T / 8 - 1) / (RK2_T / 8), C.N);
    if (C.sens_fp32) {
        if (wind)
            hipLaunchKernelGGL((k_rk4_sens2<DualF2, float, true>), grid2, dim3(RK2_T), 0, s, P, B, C.N, C.M, C.h, X,
                               U, AB, DEF, wind);
        else
            hipLaunchKernelGGL((k_rk4_sens2<DualF2, float>), grid2, dim3(RK2_T), 0, s, P, B, C.N, C.M, C.h, X, U,
                               AB, DEF, nullptr);
        hipLaunchKernelGGL(k_defects, dim3((B * C.N + 63) / 64), dim3(64), 0, s, P, B, C.N, C.M, C.h, X, U, DEF,
                           wind);
    } else if (!wind && B <= RK1_MAXB) {
        hipLaunchKernelGGL(k_rk4_sens1, dim3((B + RK1_T / 16 - 1) / (RK1_T / 16), C.N), dim3(RK1_T), 0, s, P, B,
                           C.N, C.M, C.h, X, U, AB, DEF);
    } else {
        if (wind)
            hipLaunchKernelGGL((k_rk4_sens2<Dual2, double, true>), grid2, dim3(RK2_T), 0, s, P, B, C.N, C.M, C.h, X,
                               U, AB, DEF, wind);
        else
            hipLaunchKernelGGL((k_rk4_sens2<Dual2, double>), grid2, dim3(RK2_T), 0, s, P, B, C.N, C.M, C.h, X, U,
                               AB, DEF, nullptr);
    }
    return hipGetLastError();
}
hipError_t launch_condense(const RtiConst& C, int B, const double* X, const double* U, const double* AB,
                           const double* DEF, double* Hs, double* hs, double* Cr, double* cl, double* cu,
                           double* hmax, int tiled, double* Htl, double* Hab, double* Hbb, hipStream_t s) {
    if (tiled && C.N == CD20_N && C.n == CD20_n) {
        hipLaunchKernelGGL(k_condense20, dim3(B), dim3(64), 0, s, C, B, X, U, AB, DEF, hs, Cr, cl, cu, hmax, Htl,
                           Hab, Hbb);
        return hipGetLastError();
    }
    const int NR = (C.n + 1 + 15) / 16;
#define KITE_CONDENSE(R)                                                                                    \
    case R:                                                                                                 \
        hipLaunchKernelGGL(k_condense<R>, dim3(B), dim3(64 * CondenseGeom<R>::NW), 0, s, C, B, X, U, AB, DEF, \
                           Hs, hs, Cr, cl, cu,                                                              \
                           hmax, tiled, Htl, Hab, Hbb);                                                     \
        break;
    switch (NR) {
        KITE_CONDENSE(1) KITE_CONDENSE(2) KITE_CONDENSE(3) KITE_CONDENSE(4) KITE_CONDENSE(5) KITE_CONDENSE(6)
        KITE_CONDENSE(7) KITE_CONDENSE(8) KITE_CONDENSE(9) KITE_CONDENSE(10) KITE_CONDENSE(11)
        default: return hipErrorInvalidValue;
    }
#undef KITE_CONDENSE
    return hipGetLastError();
}
hipError_t launch_qp(const ModelConst& P, const RtiConst& C, int B, const double* Hs, const double* hs,
                     const double* Cr, const double* cl, const double* cu, const double* hmax,
                     const double* AB, const double* DEF, double* X, double* U, double* u0, double* diag,
                     int32_t* status, double* kkt, int32_t* iters, const int32_t* order, int32_t* lazy,
                     hipStream_t s, hipEvent_t after_main) {
    const int G = B < QP_LAZY_GRID ? B : QP_LAZY_GRID;
    if (C.n <= 82) {
        hipLaunchKernelGGL((k_qp<82>), dim3(B), dim3(64), 0, s, P, C, B, Hs, hs, Cr, cl, cu, hmax, AB, DEF, X,
                           U, u0, diag, status, kkt, iters, order, lazy);
        if (after_main) { const hipError_t er = hipEventRecord(after_main, s); if (er != hipSuccess) return er; }
        hipLaunchKernelGGL((k_qp_lazy<82>), dim3(G), dim3(64), 0, s, P, C, B, Hs, hs, Cr, cl, cu, hmax, AB, DEF, X,
                           U, u0, diag, status, kkt, iters, order, lazy);
    } else if (C.n <= 162) {
        hipLaunchKernelGGL((k_qp<162>), dim3(B), dim3(64), 0, s, P, C, B, Hs, hs, Cr, cl, cu, hmax, AB, DEF,
                           X, U, u0, diag, status, kkt, iters, order, lazy);
        if (after_main) { const hipError_t er = hipEventRecord(after_main, s); if (er != hipSuccess) return er; }
        hipLaunchKernelGGL((k_qp_lazy<162>), dim3(G), dim3(64), 0, s, P, C, B, Hs, hs, Cr, cl, cu, hmax, AB, DEF,
                           X, U, u0, diag, status, kkt, iters, order, lazy);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
// Dispatch order of the QP grid: kites by their previous step's IPM iteration
// count, most first (a counting sort in one block; the order inside a count
// is arbitrary and never affects a result -- every kite's QP is independent).
// The QP waves run 4 per SIMD in sequence at B = 4096; dispatching the long
// ones first (largest-processing-time-first list scheduling) keeps the short
// ones for the tail, where otherwise SIMDs idle while a late long kite ends.
__global__ __launch_bounds__(1024) void k_qp_order(int B, int K, const int32_t* __restrict__ iters,
                                                   int32_t* __restrict__ order, int32_t* __restrict__ lazy) {
    __shared__ int cnt[257];
    const int t = threadIdx.x;
    if (t == 0) { lazy[0] = 0; lazy[B + 1] = 0; }     // and the prologue's cold list after it
    const int nb = (K < 255 ? K : 255) + 1;
    for (int i = t; i <= nb; i += 1024) cnt[i] = 0;
    __syncthreads();
    auto key = [&](int b) { const int v = iters[b]; return nb - 1 - (v < 0 ? 0 : (v > nb - 1 ? nb - 1 : v)); };
    for (int b = t; b < B; b += 1024) atomicAdd(&cnt[key(b)], 1);
    __syncthreads();
    if (t == 0) {
        int acc = 0;
        for (int i = 0; i < nb; ++i) { const int c = cnt[i]; cnt[i] = acc; acc += c; }
    }
    __syncthreads();
    for (int b = t; b < B; b += 1024) order[atomicAdd(&cnt[key(b)], 1)] = b;
}
// kite_nmpc_step_device's outputs in one launch instead of one copy each:
// blockIdx.y picks the array (u0, traj, ctrl, diag as doubles, status as
// 32-bit words), a grid-stride loop copies it (a null destination is skipped)
struct PublishArgs {
    const void* src[5];
    void* dst[5];
    size_t words[5];      // 8-byte words (status: 4-byte words)
};
__global__ __launch_bounds__(256) void k_publish(PublishArgs a) {
    const int y = blockIdx.y;
    if (!a.dst[y]) return;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (y < 4) {
        const double* __restrict__ src = static_cast<const double*>(a.src[y]);
        double* __restrict__ dst = static_cast<double*>(a.dst[y]);
        for (; i < a.words[y]; i += stride) dst[i] = src[i];
    } else {
        const int32_t* __restrict__ src = static_cast<const int32_t*>(a.src[y]);
        int32_t* __restrict__ dst = static_cast<int32_t*>(a.dst[y]);
        for (; i < a.words[y]; i += stride) dst[i] = src[i];
    }
}
hipError_t launch_publish(int B, int N, const double* u0, const double* X, const double* U, const double* diag,
                          const int32_t* status, double* d_u0, double* d_traj, double* d_ctrl, double* d_diag,
                          int32_t* d_status, hipStream_t s) {
    PublishArgs a;
    a.src[0] = u0; a.dst[0] = d_u0; a.words[0] = (size_t)B * 4;
    a.src[1] = X; a.dst[1] = d_traj; a.words[1] = (size_t)B * (N + 1) * 15;
    a.src[2] = U; a.dst[2] = d_ctrl; a.words[2] = (size_t)B * N * 4;
    a.src[3] = diag; a.dst[3] = d_diag; a.words[3] = (size_t)B * 6;
    a.src[4] = status; a.dst[4] = d_status; a.words[4] = (size_t)B;
    if (!d_u0 && !d_traj && !d_ctrl && !d_diag && !d_status) return hipSuccess;
    // the trajectory (B (N+1) 15 words) sets the grid: ~4 words per thread
    const size_t big = a.words[1];
    const unsigned gx = (unsigned)std::min<size_t>(std::max<size_t>((big + 1023) / 1024, 1), 4096);
    hipLaunchKernelGGL(k_publish, dim3(gx, 5), dim3(256), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_qp_order(const RtiConst& C, int B, const int32_t* iters, int32_t* order, int32_t* lazy,
                           hipStream_t s) {
    hipLaunchKernelGGL(k_qp_order, dim3(1), dim3(1024), 0, s, B, C.K, iters, order, lazy);
    return hipGetLastError();
}
hipError_t launch_dynamics(const ModelConst& P, int count, const double* x, const double* u, double* f,
                           hipStream_t s) {
    hipLaunchKernelGGL(k_dynamics, dim3((count + 63) / 64), dim3(64), 0, s, P, count, x, u, f);
    return hipGetLastError();
}
hipError_t launch_jacobian(const ModelConst& P, int count, const double* x, const double* u, double* Jx,
                           double* Ju, hipStream_t s) {
    hipLaunchKernelGGL(k_jacobian, dim3((count * 16 + 255) / 256), dim3(256), 0, s, P, count, x, u, Jx, Ju);
    return hipGetLastError();
}
hipError_t launch_predict(const ModelConst& P, int count, const double* x, const double* u, double h,
                          int steps, double* xo, hipStream_t s) {
    hipLaunchKernelGGL(k_predict, dim3((count + 63) / 64), dim3(64), 0, s, P, count, x, u, h, steps, xo);
    return hipGetLastError();
}
hipError_t launch_rk4_sens_items(const ModelConst& P, int sens_fp32, int count, int M, double h, const double* x,
                                 const double* u, double* xo, double* A, double* Bm, double* X2, double* AB,
                                 double* DEF, hipStream_t s) {
    hipLaunchKernelGGL(k_sens_items_stage, dim3((count * 2 * NX + 63) / 64), dim3(64), 0, s, count, x, X2);
    RtiConst C{};
    C.N = 1; C.M = M; C.h = h; C.sens_fp32 = sens_fp32;
    hipError_t e = launch_rk4_sens(P, C, count, X2, u, AB, DEF, nullptr, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_sens_items_expand, dim3((count * NX + 63) / 64), dim3(64), 0, s, count, M, h, x, u, AB, DEF,
                       xo, A, Bm);
    return hipGetLastError();
}
hipError_t launch_closest_point(const RtiConst& C, int count, const double* pos, const double* guess,
                                double* theta, hipStream_t s) {
    hipLaunchKernelGGL(k_closest_point, dim3((count + 63) / 64), dim3(64), 0, s, C, count, pos, guess, theta);
    return hipGetLastError();
}

#include "qp_tiled.inc"

}  // namespace kite
