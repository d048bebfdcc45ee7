/*
 * kite_nmpc.h -- C ABI of the MI355X-native batched kite NMPC (RTI) library.
 *
 * This is the drop-in boundary for openKITE's NMPC hot path.  Each entry
 * point names the reference interface it replaces (paths relative to the
 * openKITE repository).  The reference exchanges casadi::DM objects; here
 * every matrix is a plain row-major double array, batched over independent
 * NMPC instances ("batch" B).  No torch / HIP types appear in the signatures
 * except an opaque stream handle (void*).
 *
 * Conventions
 *   - Return 0 (KITE_OK) on success, a negative KITE_E* code otherwise.
 *     Per-instance solver trouble never fails a call: it is reported in the
 *     int32 status word of that instance (KITE_ST_* bits).
 *   - "host" entry points take host pointers and copy in/out (synchronous).
 *     "_device" entry points take device pointers and are asynchronous on the
 *     context stream (kite_nmpc_set_stream).
 *   - One context per host thread; a context is not re-entrant.  Contexts on
 *     different devices are independent (that is how the batch shards over
 *     GPUs: one process and one context per GPU).
 *   - There is no CPU fallback: kite_nmpc_create fails with KITE_ENODEV when
 *     no gfx950 device is usable.
 *
 * Time ordering: arrays run FORWARD in time (node 0 = t0).  The reference's
 * Chebyshev nodes run backwards (node N = t0, chebyshev.hpp:119-127,
 * kiteNMPF.cpp:232-235); the C++ facade KiteNMPF.hpp restores that column
 * order for getOptimalControl()/getOptimalTrajetory().
 */
#ifndef KITE_NMPC_H
#define KITE_NMPC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KITE_NMPC_API_VERSION 7   /* 2: kite_nmpc_config gained qp_soft_weight, qp_lm;
                                      qp_kernel 3 (multiple-shooting QP, Riccati IPM);
                                   3: kite_nmpc_config gained path_harmonics, path_fourier
                                      (arbitrary closed paths); delay_steps default 16;
                                   4: kite_nmpc_state_bound_stats (no config change);
                                   5: kite_nmpc_set_wind (no config change);
                                   6: kernel_times / timing_read report a sixth
                                      entry, the main QP kernel alone;
                                   7: kite_nmpc_timing_start_sampled (events on
                                      every stride-th step; no config change) */
#define KITE_PATH_MAX_HARMONICS 8 /* Fourier path: harmonics per axis              */

/* ---- error codes ------------------------------------------------------ */
#define KITE_OK        0
#define KITE_EINVAL   (-1)   /* bad argument                                  */
#define KITE_EHIP     (-2)   /* HIP runtime error                             */
#define KITE_ENOMEM   (-3)   /* device or host allocation failed              */
#define KITE_ENODEV   (-4)   /* no usable gfx950 device                       */
#define KITE_EIO      (-5)   /* parameter file cannot be read                 */
#define KITE_EPARSE   (-6)   /* parameter file lacks a key / bad number       */
#define KITE_ESTATE   (-7)   /* call not valid in this context state          */

/* ---- per-instance status bits (status_out) ---------------------------- */
#define KITE_ST_NAN            1   /* non-finite value in the new iterate     */
#define KITE_ST_QP_NOT_CONV    2   /* QP residual > 1e-8 after the cap K       */
#define KITE_ST_MIN_SPEED      4   /* vx clamped to min_speed (nmpf_node.cpp:241-243) */
#define KITE_ST_STATE_BOUND    8   /* new trajectory still outside lbx/ubx after the
                                      lazy state-bound rows (vx: a QP row at every
                                      node; states 1..12: at most 4 rows per step,
                                      2 re-solves -- DESIGN.md 4.4)                */
#define KITE_ST_THETA_WRAP    16   /* theta wrapped by 2*pi (kiteNMPF.cpp:212-221) */
#define KITE_ST_STEP_REJECTED 32   /* QP residual >= 1e-6 or NaN: no step applied, the
                                      shifted plan is kept (the reference applies the
                                      failed iterate, kiteNMPF.cpp:303-313)          */
#define KITE_ST_RESTART       64   /* the warm start held non-finite values: this kite
                                      was restarted cold, theta from the closest point
                                      and thetadot = 0 (nmpf_node.cpp:225-236)        */

/* ---- model parameters: kite_utils::LoadProperties (kite.cpp:7-76) ------
 * Field order == KiteProperties (kite.h:9-93) flattened.  52 doubles.     */
typedef struct kite_params {
    /* geometry */
    double b, c, AR, S, lam, St, lt, Sf, lf, Xac;
    /* inertia */
    double mass, Ixx, Iyy, Izz, Ixz;
    /* aerodynamics */
    double CL0, CL0_tail, CLa_total, CLa_wing, CLa_tail, e_oswald;
    double CD0_total, CD0_wing, CD0_tail, CYb, CYb_vtail, Cm0, Cma;
    double Cn0, Cnb, Cl0, Clb, CLq, Cmq, CYr, Cnr, Clr, CYp, Clp, Cnp;
    double CLde, CYdr, Cmde, Cndr, Cldr, CDde;
    /* tether */
    double Lt, Ks, Kd, rx, ry, rz;
} kite_params;

/* ---- controller configuration ------------------------------------------
 * Replaces the KiteNMPF ctor + setters + createNLP (kiteNMPF.h:14-37,
 * kiteNMPF.cpp:18-197) and the values the ROS node feeds them
 * (nmpf_node.cpp:30-69).  Units are physical; Sx/Su are the diagonals of the
 * reference scaling matrices (setStateScaling / setControlScaling).      */
typedef struct kite_nmpc_config {
    int32_t N;            /* shooting intervals (20; 40 for long horizons)     */
    int32_t M;            /* RK4 substeps per interval (2)                     */
    int32_t qp_iters;     /* interior-point iteration cap K (16)               */
    int32_t shift;        /* 1: shift the warm start by one interval per step  */
    int32_t device;       /* HIP device ordinal                                 */
    int32_t timing;       /* 1: record per-kernel hipEvents (kite_nmpc_kernel_times) */
    int32_t qp_kernel;    /* 0: auto (2 at N == 20, else 3), 1: condensed QP, wave-scalar LDS IPM,
                             2: condensed QP, MFMA-tiled IPM (register tiles at N == 20, LDS
                             tiles with 4 waves per kite at N == 40; KITE_EINVAL otherwise),
                             3: multiple-shooting QP (every node state a variable, as the
                             reference NLP kiteNMPF.cpp:145-160), Riccati IPM on MFMA tiles,
                             soft state bounds (qp_soft_weight) and a Levenberg-Marquardt
                             term (qp_lm).  1 and 2 enforce the state bounds of states 1..12
                             as lazy rows. */
    int32_t delay_steps;  /* RK4 substeps of the delay-compensation prediction (16) */
    double dt;            /* interval length [s] (0.05 -> tf = 1 s at N = 20)  */
    double Q[3];          /* path weights  (kiteNMPF.cpp:32)                   */
    double R[4];          /* control weights (kiteNMPF.cpp:33)                 */
    double W;             /* path-speed weight (kiteNMPF.cpp:34)               */
    double Sx[15], Su[4]; /* scaling diagonals (nmpf_node.cpp:50-51)           */
    double lbx[15], ubx[15];  /* state bounds (nmpf_node.cpp:59-63); +-INFINITY = none;
                                 13, 14 (theta, thetadot) are not bounded    */
    double lbu[4], ubu[4];    /* control bounds (nmpf_node.cpp:45-47)          */
    double vref;          /* physical path speed (setReferenceVelocity, nmpf_node.cpp:68) */
    double path_radius;   /* P(theta) = rot(q)[R cos, R sin, alt] (nmpf_node.cpp:30-40)
                             when path_harmonics == 0 (see path_fourier)             */
    double path_altitude;
    double path_q[4];     /* (w,x,y,z); P = vec(q^-1 (x) p (x) q)               */
    double theta_flex;    /* +- relaxation of theta, thetadot at t0 (kiteNMPF.cpp:226) */
    double min_speed;     /* caller-side vx clamp (nmpf_node.cpp:241-243); <= -INF disables */
    double delay;         /* transport-delay compensation of the ROS node, fused into
                             the step (nmpf_node.cpp:206-221): on warm steps the kite
                             part of x0 is predicted over `delay` s under the previous
                             u(t0) (RK4, delay_steps substeps; the node used CVODES,
                             abstol 1e-4: 16 substeps stay within 2e-5)
                             and theta, thetadot are taken from the previous trajectory
                             at node round(delay/dt).  0 = off: KiteNMPF semantics, the
                             caller passes the predicted state (default).  The node
                             uses 0.1 (nmpf_node.cpp:74).                              */
    int32_t sens_fp32;    /* 1: RK4 + forward sensitivities in fp32 (mixed precision,
                             BASELINE config 4); condensing, QP, expansion stay fp64 */
    int32_t reserved;
    double qp_soft_weight; /* qp_kernel 3: exact-L1 weight of the state bounds in the reference's
                              scaled units (1e3); the QP stays feasible when the linearised
                              dynamics cannot meet the box over the horizon.  Must exceed
                              40 = 2 z0 (the IPM's start multiplier, so every soft row starts
                              dual feasible): smaller values give KITE_EINVAL                 */
    double qp_lm;          /* qp_kernel 3: Levenberg-Marquardt term lm/2 ||step||^2 on every QP
                              variable, scaled units (10); leaves the RTI fixed point unchanged.
                              qp_lm = 0 with qp_soft_weight = 1e6 at N = 20: the condensed
                              QP's own step with the state box exact on every node
                              (DESIGN.md 4.4); at N = 40 the undamped step diverges        */
    /* Arbitrary closed path (KiteNMPF(kite, path), kiteNMPF.h:14, takes any
     * casadi::Function theta -> R^3): with path_harmonics = K in 1..8 the
     * unrotated curve is the truncated Fourier series
     *   p_a(theta) = F[a][0] + sum_{k=1..K} F[a][2k-1] cos(k theta) + F[a][2k] sin(k theta)
     * per axis a = x, y, z, and P(theta) = vec(q^-1 (x) [0, p] (x) q) with path_q
     * as for the circle (path_radius / path_altitude are then unused).  The
     * circle is K = 1, F[0][1] = F[1][2] = R, F[2][0] = alt.  0 (default): the
     * circle.  Every path evaluation of the step (closest point, residuals,
     * diagnostics, kite_nmpc_path_eval) uses it.                               */
    int32_t path_harmonics;
    int32_t reserved2;
    double path_fourier[3][2 * KITE_PATH_MAX_HARMONICS + 1];
} kite_nmpc_config;

/* ---- diagnostics: msg/mpc_diagnostic.msg (filled at nmpf_node.cpp:191-204) */
typedef struct kite_mpc_diagnostic {
    double pos_error;     /* ||Sr (P(theta0) - r0)||  (kiteNMPF.cpp:319-330)    */
    double vel_error;     /* |Sx14 (vref - thetadot0)| (kiteNMPF.cpp:333-344)   */
    double cost;          /* objective of the new iterate (reference sends 0)  */
    double virt_state;    /* theta at t0 (kiteNMPF.cpp:347-355)                 */
    double virt_ctrl;     /* Uv at t0 (unset in the reference)                  */
    double comp_time_ms;  /* host-measured step time of the whole batch         */
} kite_mpc_diagnostic;

typedef struct kite_nmpc_ctx kite_nmpc_ctx;

/* kite_utils::LoadProperties (kite.cpp:7-76).  Unlike the reference, a
 * missing tether.rx/ry/rz defaults to 0 (the shipped umx_radian.yaml lacks
 * them); any other missing key is KITE_EPARSE.              */
int kite_params_load_yaml(const char* path, kite_params* out);

/* Node defaults: nmpf_node.cpp:30-69 + kiteNMPF.cpp:32-34 + RTI settings.  */
void kite_nmpc_default_config(kite_nmpc_config* cfg);

/* KiteNMPF ctor + setters + createNLP (kiteNMPF.cpp:18-197).  Allocates all
 * device buffers for `batch` instances on cfg->device.                      */
int kite_nmpc_create(const kite_params* params, const kite_nmpc_config* cfg,
                     int32_t batch, kite_nmpc_ctx** out);
void kite_nmpc_destroy(kite_nmpc_ctx* ctx);
const char* kite_nmpc_strerror(int code);

/* setLBX/setUBX/setLBU/setUBU (kiteNMPF.h:20-27).  NULL keeps a vector.     */
int kite_nmpc_set_bounds(kite_nmpc_ctx* ctx, const double* lbx15, const double* ubx15,
                         const double* lbu4, const double* ubu4);
/* setReferenceVelocity (kiteNMPF.h:34); physical units.                     */
int kite_nmpc_set_reference_velocity(kite_nmpc_ctx* ctx, double vref);
/* disableWarmStart (kiteNMPF.h:40): the next step cold-starts.              */
int kite_nmpc_reset(kite_nmpc_ctx* ctx);
/* Wind-field sweeps (the batch dimension of BASELINE north_star): a constant
 * world-frame wind per instance, wind[3 b + i] in m/s (B x 3), or NULL for
 * none.  Build extension: the reference model has no wind (kite.cpp:196
 * "@todo: add wind"); with wind the RTI model's aerodynamics see the
 * air-relative velocity v - q^-1 W q (kite_model.hpp), used by every step's
 * prediction (cold start, delay compensation, sensitivities, defects).  The
 * item-wise model entry points (dynamics, jacobian, predict, rk4_sens) and
 * the EKF keep the reference model.  All-zero wind is the reference model
 * bit for bit.  Non-finite entries: KITE_EINVAL.                            */
int kite_nmpc_set_wind(kite_nmpc_ctx* ctx, const double* wind);
/* Run on this HIP stream (hipStream_t as void*).  NULL is the HIP null
 * (legacy default) stream -- the stream PyTorch's default stream maps to.
 * A new context runs on a private non-blocking stream; restore it with
 * kite_nmpc_use_own_stream.                                                  */
int kite_nmpc_set_stream(kite_nmpc_ctx* ctx, void* hip_stream);
int kite_nmpc_use_own_stream(kite_nmpc_ctx* ctx);
int kite_nmpc_synchronize(kite_nmpc_ctx* ctx);

/* findClosestPointOnPath (kiteNMPF.cpp:358-391), batched over `count`
 * positions (count x 3); guess may be NULL (= 0 as in the reference).       */
int kite_nmpc_closest_point(kite_nmpc_ctx* ctx, int32_t count, const double* pos,
                            const double* guess, double* theta_out);
/* getPathFunction (kiteNMPF.h:46; the path built at nmpf_node.cpp:30-40 and
 * evaluated per trajectory node for /opt_traj at nmpf_node.cpp:177-183):
 * P(theta) = vec(q^-1 (x) [0, p(theta)] (x) q) (the circle p = [R cos, R sin,
 * alt] or the Fourier curve of path_harmonics) and dP/dtheta for
 * `count` angles (count x 3 each; dP3 may be NULL).  Host arithmetic on the
 * configuration only (no context, no GPU): a visualisation helper of the
 * node, not part of the RTI step.                                           */
int kite_nmpc_path_eval(const kite_nmpc_config* cfg, int32_t count, const double* theta,
                        double* P3, double* dP3);

/* One RTI step for the whole batch: replaces KiteNMPF::computeControl
 * (kiteNMPF.cpp:199-316) -- NLP_Solver(ARG) becomes shift -> rk4_sens ->
 * condense -> QP -> expand.
 *   x0        B x 15 augmented state [v w r q theta thetadot] (physical)
 *   u0_out    B x 4  control to apply = last column of getOptimalControl()
 *   traj_out  B x (N+1) x 15 optimal trajectory (forward time), nullable
 *   ctrl_out  B x N x 4 optimal controls, nullable
 *   diag_out  B mpc_diagnostic records, nullable
 *   status_out B status words, nullable                                      */
int kite_nmpc_step(kite_nmpc_ctx* ctx, const double* x0, double* u0_out,
                   double* traj_out, double* ctrl_out, kite_mpc_diagnostic* diag_out,
                   int32_t* status_out);
/* Same, device pointers, asynchronous on the context stream.  diag_out is
 * B x 6 doubles in kite_mpc_diagnostic order (comp_time_ms left 0).          */
int kite_nmpc_step_device(kite_nmpc_ctx* ctx, const double* d_x0, double* d_u0,
                          double* d_traj, double* d_ctrl, double* d_diag, int32_t* d_status);

/* Warm-start access (getOptimalTrajetory / getOptimalControl state, and
 * NLP_X warm start injection).  Host pointers, B x (N+1) x 15 and B x N x 4. */
int kite_nmpc_get_solution(kite_nmpc_ctx* ctx, double* traj, double* ctrl);
int kite_nmpc_set_solution(kite_nmpc_ctx* ctx, const double* traj, const double* ctrl);

/* ---- model-level entry points (KiteDynamics, kite.cpp:320-338) ---------- */
/* getNumericDynamics: f(x,u), count x 15 states (augmented), count x 4 ctrl. */
int kite_nmpc_dynamics(kite_nmpc_ctx* ctx, int32_t count, const double* x15,
                       const double* u4, double* f15);
/* getNumericJacobian: df/dx (13 x 13) and df/du (13 x 3) of the kite ODE.    */
int kite_nmpc_jacobian(kite_nmpc_ctx* ctx, int32_t count, const double* x13,
                       const double* u3, double* Jx, double* Ju);
/* RK4 integrator (kitemath.cpp:36-51, integrator.cpp:86-98) with `steps`
 * substeps over tf: the delay-compensation predictor of nmpf_node.cpp:218.   */
int kite_nmpc_predict(kite_nmpc_ctx* ctx, int32_t count, const double* x15,
                      const double* u4, double tf, int32_t steps, double* x15_out);
/* The hot kernel alone (k_rk4_sens2 on `count` one-interval horizons, BASELINE
 * config 2): x+ and S = dx+/d[x,u] over one shooting interval (h = tf/M, M
 * substeps).  count x 15, count x 4 -> count x 15, count x 15 x 15,
 * count x 15 x 4.  Sensitivities in fp32 (x+ in fp64) when the context was
 * created with config.sens_fp32 = 1.                                        */
int kite_nmpc_rk4_sens(kite_nmpc_ctx* ctx, int32_t count, const double* x15,
                       const double* u4, double tf, int32_t M, double* xnext,
                       double* A, double* B);

/* ---- introspection (tests, profiling) ---------------------------------- */
/* ---- reference formulation: Chebyshev collocation (chebyshev.hpp) -------
 * Evaluates the reference's own NLP functions for `count` points
 * z = [X (nodes x 15) | U (nodes x 4)], nodes = poly_order*num_segments + 1,
 * in the reference's (optionally scaled) variables:
 *   G = (CompDiff (x) I15) X - t_scale * SODE(X_i, U_i)      (chebyshev.hpp:241-271)
 *   J = mayer_scale * M(X_0) + sum_seg t_scale sum_m w_m L(X, U) (:280-333)
 * with t_scale = (tf - t0) / (2 num_segments), SODE(x, u) = Sx f_aug(x/Sx, u/Su)
 * (kiteNMPF.cpp:100-104), L = Q.res^2 + W (vref - x14)^2 [+ R.u^2],
 * res = Sx_r P(x13 / Sx13) - x(6:9), M = Q.res^2 (kiteNMPF.cpp:117-143).
 * jac (nullable): per node the 15 x 19 block d SODE / d [x, u] at (X_i, U_i);
 * the constraint Jacobian is dG/dX = CompDiff (x) I - t_scale blockdiag(jac_x),
 * dG/dU = -t_scale blockdiag(jac_u).                                         */
typedef struct kite_colloc_config {
    int32_t poly_order;     /* 5 (kiteNMPF.cpp:83); 10 in full_generics_test     */
    int32_t num_segments;   /* 2 (kiteNMPF.cpp:82); 1 in full_generics_test      */
    int32_t use_R;          /* 1: L includes R u^2 (NMPF); 0: full_generics_test */
    int32_t reserved;
    double t0, tf;
    double Q[3], R[4], W;
    double vref;            /* in the formulation's variables (Sx14 * v when scaled) */
    double mayer_scale;     /* 1 (NMPF), 2 (full_generics_test)                   */
    double Sx[15], Su[4];   /* 1 = unscaled                                       */
    double path_radius, path_altitude, path_q[4];
    int32_t path_harmonics;  /* as kite_nmpc_config (API 3): 0 the circle, 1..8 Fourier path */
    int32_t reserved2;
    double path_fourier[3][2 * KITE_PATH_MAX_HARMONICS + 1];
} kite_colloc_config;
/* The NMPF's setup (kiteNMPF.cpp:80-143 with the node's scaling and path).  */
void kite_colloc_default_config(kite_colloc_config* cfg);
int kite_nmpc_colloc_eval(kite_nmpc_ctx* ctx, const kite_colloc_config* cfg, int32_t count, const double* z,
                          double* G, double* J, double* jac);

/* ---- extended Kalman filter: KiteEKF (src/kite_estimation/kiteEKF.cpp) ---
 * For each of `count` kites: propagate(dt) (kiteEKF.cpp:75-98: one RK4 step,
 * A = I + J dt, P = A P A' + W) and, when z7 != NULL, the update of
 * _estimate (kiteEKF.cpp:108-126) with H = [0_{7x6} I_7] (position r and
 * quaternion q measured).  x13 (count x 13) and P169 (count x 13 x 13,
 * row-major) are updated in place; u3 count x 3 (T, dE, dR); z7 count x 7;
 * W169 / V49 shared by all kites.                                           */
void kite_ekf_default_covariances(double* W169, double* V49, double* P0_169);  /* kiteEKF.cpp:6-13,26 */
int kite_nmpc_ekf_step(kite_nmpc_ctx* ctx, int32_t count, double dt, double* x13, const double* u3,
                       double* P169, const double* z7, const double* W169, const double* V49);
/* Same on device pointers, asynchronous on the context stream.              */
int kite_nmpc_ekf_step_device(kite_nmpc_ctx* ctx, int32_t count, double dt, double* d_x13,
                              const double* d_u3, double* d_P169, const double* d_z7,
                              const double* d_W169, const double* d_V49);

/* Per-kernel device time [ms] of the last step (cfg.timing = 1):
 * [prologue, rk4_sens, condense, qp, total, qp_main]; qp is the whole QP
 * phase (solve, expansion, lazy state rows), qp_main the main QP kernel
 * alone (k_qp_tiled / k_qp_lds / k_qp / k_qp_ric: the roofline's kernel).
 * Returns the entries written, min(n, 6).                                   */
int kite_nmpc_kernel_times(kite_nmpc_ctx* ctx, double* ms, int32_t n);
/* Time every kernel of the next max_steps steps with a ring of HIP events
 * (no host synchronisation between steps); timing_read waits for the last
 * recorded step and returns the number of steps recorded, with per-kernel
 * SUMS [ms] in the first min(n, 6) entries of sums_ms:
 * [prologue, rk4_sens, condense, qp, total, qp_main] (as kernel_times).   */
int kite_nmpc_timing_start(kite_nmpc_ctx* ctx, int32_t max_steps);
/* The same ring, recording only every stride-th step from the next one on
 * (steps 0, stride, 2 stride, ...), at most max_samples of them; timing_read
 * returns the number recorded.  Each recorded step places six events between
 * its kernels (~4.6 us each on gfx950); sampling keeps that measurement cost
 * out of the other steps of a timed run.  stride 1 = kite_nmpc_timing_start
 * (since API 7).                                                           */
int kite_nmpc_timing_start_sampled(kite_nmpc_ctx* ctx, int32_t max_samples, int32_t stride);
int kite_nmpc_timing_read(kite_nmpc_ctx* ctx, double* sums_ms, int32_t n);
/* QP statistics of the last step: final residual and interior-point
 * iterations per instance (host pointers, B each; either may be NULL).    */
int kite_nmpc_qp_stats(kite_nmpc_ctx* ctx, double* kkt, int32_t* iters);
/* Interior-point iterations summed over all instances and all steps since
 * the last kite_nmpc_timing_start (or since create): the measurement hook
 * behind bench.py's FLOP count (no reference counterpart).                */
int kite_nmpc_qp_iteration_sum(kite_nmpc_ctx* ctx, int64_t* sum);
/* State-box enforcement since the last kite_nmpc_timing_start (or since
 * create), summed over instances and steps: kite-steps whose committed plan
 * leaves the state box (status bit 8) and the (node, state) pairs outside it
 * (states 1..12, nodes 1..N, tolerance 1e-8 max(1, |bound|)); with the
 * multiple-shooting QP the latter are the soft rows with xi > 0 at the
 * accepted solution.  The reference's NLP holds these as hard bounds
 * (kiteNMPF.cpp:154-167); measurement hook, either pointer may be NULL.    */
int kite_nmpc_state_bound_stats(kite_nmpc_ctx* ctx, int64_t* steps_outside, int64_t* rows_outside);
/* Condensed QP of one instance from the last step (scaled variables, GPU
 * column order: [T,dE,dR]_k (3N) | Uv_k (N) | theta0 | thetadot0).
 * H n x n, h n, C N x n, cl/cu N (+-INF = absent), n = 4N+2.               */
int kite_nmpc_get_qp(kite_nmpc_ctx* ctx, int32_t instance, double* H, double* h,
                     double* C, double* cl, double* cu);
int kite_nmpc_batch(const kite_nmpc_ctx* ctx);
int kite_nmpc_api_version(void);

#ifdef __cplusplus
}
#endif
#endif /* KITE_NMPC_H */
