// rti_kernels.hpp -- internal interface between the C ABI (kite_nmpc.cpp) and
// the gfx950 kernels (rti_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kite_model.hpp"
#include "kite_path.hpp"

// Largest horizon the fused condense/QP kernels are built for (LDS budget of
// the wave-per-instance QP).  n = 4N+2 <= 82 decision variables.
#define KITE_NMAX 40

namespace kite {

// Everything the RTI kernels need besides the model, precomputed on the host
// from kite_nmpc_config (kernel argument, < 1 KiB).
struct RtiConst {
    int N, M, K, n;
    int shift, lo_fin, hi_fin, pad_;
    double dt, h;
    double sqQ_dt[3];   // sqrt(dt Q_i)   stage path weights
    double sqQ_T[3];    // sqrt(Q_i)      Mayer path weights (kiteNMPF.cpp:141)
    double sw;          // sqrt(dt W)
    double Sr[3];       // Sx[6..8]
    double sv;          // Sx[14]
    double vref;        // physical
    double Rdiag[4];    // dt R_c Su_c^2
    double Rraw[4];     // R_c
    double Su[4], Sx13, Sx14;
    double lbx[15], ubx[15], lbu[4], ubu[4];
    double flex, min_speed;
    double path_R, path_alt, pq[4];
    double delay;       // delay compensation [s] (0 = off)
    int delay_steps, delay_node;
    int sens_fp32, pad2_;   // 1: k_rk4_sens2 in fp32 (DualF2)
    int path_K, pad3_;      // 0: circle (path_R, path_alt); 1..8: Fourier path pF (kite_path.hpp)
    double pF[3][KITE_PATH_NC];
};

// Start multiplier z0 of the multiple-shooting IPM (qp_ric.inc; the oracle's
// MS_Z0 holds the same value).  A soft state row starts dual feasible only if
// its weight exceeds 2 z0 (z2 = soft_w - z0 > z0): kite_nmpc_create /
// set_bounds refuse qp_soft_weight <= RIC_SOFT_WEIGHT_MIN for qp_kernel 3.
constexpr double RIC_Z0 = 20.0;
constexpr double RIC_SOFT_WEIGHT_MIN = 2.0 * RIC_Z0;

// Multiple-shooting QP + Riccati interior point (qp_ric.inc, oracle qp_form 1):
// constants precomputed on the host from kite_nmpc_config.
struct RicConst {
    double soft_w;      // L1 weight of the soft state bounds (scaled units)
    double lm;          // Levenberg-Marquardt term on every QP variable
    double hth, g0, g1; // scaled theta dynamics: th' = th + hth thd + g0 Uv, thd' = thd + g1 Uv
    double sq[2][3];    // path rows sqrt(w Q_a): [0] k < N (w = dt), [1] k = N (w = 1)
    double sw;          // speed row sqrt(dt W)
    double ctheta;      // Sx[6+a] / Sx13 factor of dP/dtheta in the theta column: 1 / Sx13
    double Rh[4];       // control Hessian (scaled): dt R_c
    double lb[20], ub[20], sc[20];   // per stage slot: bound and scale (see qp_ric.inc)
    int nC;             // complementarity pairs per kite (rows + soft rows over all stages)
    int lomask[3], himask[3];        // bit j: slot j has a lower / upper bound row at stage
                                     // type t (0: k = 0, 1: 0 < k < N, 2: k = N)
    int nb[3];                       // bounded slots per stage type ...
    int8_t bslot[3][20];             // ... and their slot numbers
};
bool qp_ric_supported(const RtiConst& C);
size_t qp_ric_lds_bytes(const RtiConst& C, const RicConst& R);
// C, R: host copies (launch geometry); Cd, Rd: the same constants in device memory;
// ws: workspace of qp_ric_ws_doubles(C) doubles per kite
size_t qp_ric_ws_doubles(const RtiConst& C);
hipError_t launch_qp_ric(const RtiConst& C, const RicConst& R, const RtiConst* Cd, const RicConst* Rd, int B,
                         const double* AB, const double* DEF, double* X, double* U, double* u0, double* diag,
                         int32_t* status, double* kkt, int32_t* iters, int32_t* iters_acc, const int32_t* order,
                         double* ws, hipStream_t s, hipEvent_t after_main = nullptr);

// wind: per-kite constant world-frame wind (B x 3, m/s) or nullptr (the
// reference model, no wind; kite_model.hpp kite_rhs<T, WIND>)
// cold: B + 1 ints, the prologue's cold-restart list (count first; zero on
// entry -- k_qp_order empties it every step)
hipError_t launch_prologue(const ModelConst& P, const RtiConst& C, int B, int warm, const double* x0,
                           double* X, double* U, int32_t* status, const double* wind, int32_t* cold,
                           hipStream_t s);
hipError_t launch_rk4_sens(const ModelConst& P, const RtiConst& C, int B, const double* X, const double* U,
                           double* AB, double* DEF, const double* wind, hipStream_t s);
hipError_t launch_condense(const RtiConst& C, int B, const double* X, const double* U, const double* AB,
                           const double* DEF, double* Hs, double* hs, double* Cr, double* cl, double* cu,
                           double* hmax, int tiled, double* Htl, double* Hab, double* Hbb, hipStream_t s);
// Tiled-QP path (N == 20): H_aa as 15 lower 16x16 C-layout tiles in lane order.
bool qp_tiled_supported(const RtiConst& C);
hipError_t launch_qp_tiled(const ModelConst& P, const RtiConst& C, int B, const double* Htl, const double* Hab,
                           const double* Hbb, const double* hs, const double* Cr, const double* cl,
                           const double* cu, const double* hmax, const double* AB, const double* DEF, double* X,
                           double* U, double* u0, double* diag, int32_t* status, double* kkt, int32_t* iters,
                           const int32_t* order, int32_t* lazy, double* wstep, hipStream_t s,
                           hipEvent_t after_main = nullptr);
hipError_t launch_qp(const ModelConst& P, const RtiConst& C, int B, const double* Hs, const double* hs,
                     const double* Cr, const double* cl, const double* cu, const double* hmax,
                     const double* AB, const double* DEF, double* X, double* U, double* u0, double* diag,
                     int32_t* status, double* kkt, int32_t* iters, const int32_t* order, int32_t* lazy,
                     hipStream_t s, hipEvent_t after_main = nullptr);
// QP grid dispatch order: kites by the previous step's iteration count, most
// first; also empties the lazy state-bound list (lazy[0] = 0, B + 1 entries)
// and the prologue's cold list that follows it (lazy[B + 1] = 0)
hipError_t launch_publish(int B, int N, const double* u0, const double* X, const double* U, const double* diag,
                          const int32_t* status, double* d_u0, double* d_traj, double* d_ctrl, double* d_diag,
                          int32_t* d_status, hipStream_t s);
hipError_t launch_qp_order(const RtiConst& C, int B, const int32_t* iters, int32_t* order, int32_t* lazy,
                           hipStream_t s);
hipError_t launch_dynamics(const ModelConst& P, int count, const double* x, const double* u, double* f,
                           hipStream_t s);
hipError_t launch_jacobian(const ModelConst& P, int count, const double* x, const double* u, double* Jx,
                           double* Ju, hipStream_t s);
hipError_t launch_predict(const ModelConst& P, int count, const double* x, const double* u, double h,
                          int steps, double* xo, hipStream_t s);
hipError_t launch_rk4_sens_items(const ModelConst& P, int sens_fp32, int count, int M, double h, const double* x,
                                 const double* u, double* xo, double* A, double* Bm, double* X2, double* AB,
                                 double* DEF, hipStream_t s);
hipError_t launch_closest_point(const RtiConst& C, int count, const double* pos, const double* guess,
                                double* theta, hipStream_t s);
// Chebyshev collocation evaluator (colloc_kernels.hip): constants of one formulation
struct CollocConst {
    int nodes, use_R;
    double t_scale, mayer_scale;
    double Q[3], R[4], W, vref;
    double Sx[15], Su[4], iSx[15], iSu[4];
    double path_R, path_alt, pq[4];
    int path_K, pad_;
    double pF[3][KITE_PATH_NC];
};
// tab = CompDiff (nodes x nodes, row-major) followed by the node weights (nodes)
hipError_t launch_colloc(const ModelConst& P, const CollocConst& C, int count, const double* tab, const double* z,
                         double* G, double* J, double* jac, hipStream_t s);
// batched EKF propagate (+ update when z != nullptr), in place on x and Pc (ekf_kernels.hip)
hipError_t launch_ekf(const ModelConst& P, int count, double dt, double* x, const double* u, double* Pc,
                      const double* z, const double* W, const double* V, hipStream_t s);

}  // namespace kite
