// kite_nmpc.cpp -- host side of the C ABI declared in include/kite_nmpc/kite_nmpc.h.
//
// Owns the device buffers of one batch of NMPC instances on one GPU and
// sequences the RTI kernels (rti_kernels.hip) on a HIP stream.  There is no
// CPU fallback: every numerical entry point runs on the GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "kite_nmpc/kite_nmpc.h"
#include "rti_kernels.hpp"

using kite::ModelConst;
using kite::RtiConst;

// HIP events per timed step: before the prologue, after the prologue, after
// rk4_sens, after condense + qp_order, after the QP phase (expansion and lazy
// rows included), and [5] after the main QP kernel alone (k_qp_tiled /
// k_qp_lds / k_qp / k_qp_ric) -- the roofline's kernel, between [3] and [5]
constexpr int KITE_NEV = 6;
// The phase events only time the step: no system-scope fence when they are
// recorded.  With the default flags every record wrote back and invalidated
// the caches, 5.6-5.9 us between the kernels it separated (six per step, 2 %
// of the headline step in profiles/r05m's trace) -- measurement overhead
// inside the timed region.  Completion is still observable: timing_read
// synchronises on the last event before reading the elapsed times, and no
// caller reads device memory through these events.
constexpr unsigned kTimingEventFlags = hipEventDisableSystemFence;

struct kite_nmpc_ctx {
    kite_params params;
    kite_nmpc_config cfg;
    int B = 0;
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    bool warm = false;
    ModelConst mc;
    RtiConst rc;
    // device buffers (see rti_kernels.hip for layouts)
    double *X = nullptr, *U = nullptr, *x0 = nullptr, *AB = nullptr, *DEF = nullptr;
    double *Hs = nullptr, *hs = nullptr, *Cr = nullptr, *cl = nullptr, *cu = nullptr, *hmax = nullptr;
    double *u0 = nullptr, *diag = nullptr, *kkt = nullptr;
    int32_t* status = nullptr;
    int32_t* iters = nullptr;
    int32_t* order = nullptr;      // QP dispatch order (k_qp_order), B entries, then the lazy
                                   // state-bound list (B + 1: count, kites), then the
                                   // prologue's cold-restart list (B + 1)
    // tiled-QP layout (N == 20, 40): H_aa lower tiles [B][NT(NT+1)/2][4][64] with
    // NT = N/4, H_ab [B][4N][2], H_bb [B][2][2]
    bool tiled = false;
    bool ric = false;              // multiple-shooting QP + Riccati IPM (qp_kernel 3): no condensing
    kite::RicConst ricc;
    // device copy of (rc, ricc) read by k_qp_ric; re-uploaded when the host copy changes
    void* dconst = nullptr;
    std::vector<unsigned char> dconst_host;     // what dconst holds (empty: unknown)
    std::vector<unsigned char> dconst_stage;
    double *Htl = nullptr, *Hab = nullptr, *Hbb = nullptr;
    double* wind = nullptr;        // per-kite world-frame wind B x 3 (kite_nmpc_set_wind)
    bool has_wind = false;         // a nonzero wind is set: the WIND kernels run
    double* wstep = nullptr;       // tiled path, 2 B n: physical QP step per kite (k_qp_tiled -> k_expand20), then
                                   // the scaled one (-> k_qp_tiled_lazy: round 0 handed over); N = 40:
                                   // round-0 solution of the kites k_qp_lds hands to k_qp_lds_lazy
    // scratch for the model-level entry points
    double* scratch = nullptr;
    size_t scratch_bytes = 0;
    hipEvent_t ev[KITE_NEV] = {};
    bool timed_step = false;
    // the prologue's cold-restart count (order + 2B + 1) is zeroed by k_qp_order
    // later in the same step; set while a step is between the two launches, so
    // a step that returned early in between zeroes it before the next prologue
    bool cold_dirty = false;
    // event ring for timing a whole run without host syncs (kite_nmpc_timing_start),
    // KITE_NEV events per step
    std::vector<hipEvent_t> ring;
    int ring_cap = 0, ring_used = 0;
    int ring_stride = 1, ring_phase = 0;   // record every ring_stride-th step
    // kite_nmpc_step's launch sequence (x0 in, every kernel of the step, the
    // outputs out) captured once per warm / cold start into a HIP graph, with
    // pinned host staging: one graph launch and one synchronisation per step
    // instead of ~10 launches and 6 pageable copies (the ROS node's batch-1
    // latency).  Captured kernels take the context constants by value, so the
    // setters that change them bump graph_gen and the graphs are re-captured.
    hipGraphExec_t gexec[2] = {nullptr, nullptr};  // [warm]
    unsigned graph_gen = 0, gexec_gen[2] = {0, 0};
    bool graph_off = false;                         // KITE_NMPC_NO_GRAPH=1 (A/B runs)
    double* h_in = nullptr;                         // pinned: B x 15
    unsigned char* h_out = nullptr;                 // pinned: u0 | traj | ctrl | diag | status
    unsigned char* d_out = nullptr;                 // device staging of the same layout
};

namespace {

int hip_fail(hipError_t e) {
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return KITE_ENOMEM;
    return KITE_EHIP;
}
#define HIP_TRY(expr)                                     \
    do {                                                  \
        hipError_t e_ = (expr);                           \
        if (e_ != hipSuccess) return hip_fail(e_);        \
    } while (0)

ModelConst make_model_const(const kite_params& p) {
    ModelConst m;
    const double rho = kite::kRho;
    m.inv_mass = 1.0 / p.mass;
    m.S = p.S; m.b = p.b; m.c = p.c;
    m.CL0 = p.CL0; m.CLa = p.CLa_total; m.CD0 = p.CD0_total;
    m.inv_pieAR = 1.0 / (3.14159265358979323846 * p.e_oswald * p.AR);   // casadi::pi
    m.kLq = 0.25 * p.CLq * p.c * p.S * rho;
    m.CYb = p.CYb; m.CYdr = p.CYdr; m.kSF = 0.25 * p.b * rho * p.S;
    m.CYr = p.CYr; m.CYp = p.CYp;
    m.CLde = p.CLde;
    m.Cl0 = p.Cl0; m.Clb = p.Clb; m.Cldr = p.Cldr; m.Clr = p.Clr; m.Clp = p.Clp;
    m.kRoll = 0.25 * rho * p.b * p.b * p.S;
    m.Cm0 = p.Cm0; m.Cma = p.Cma; m.Cmde = p.Cmde; m.Cmq = p.Cmq;
    m.kPitch = 0.25 * p.S * p.c * p.c * rho;
    m.Cn0 = p.Cn0; m.Cnb = p.Cnb; m.Cndr = p.Cndr; m.Cnp = p.Cnp; m.Cnr = p.Cnr;
    m.kYaw = 0.25 * p.S * p.b * p.b * rho;
    m.Ixx = p.Ixx; m.Iyy = p.Iyy; m.Izz = p.Izz; m.Ixz = p.Ixz;
    const double det = p.Ixx * p.Izz - p.Ixz * p.Ixz;
    m.Ji00 = p.Izz / det; m.Ji02 = -p.Ixz / det; m.Ji22 = p.Ixx / det; m.Ji11 = 1.0 / p.Iyy;
    m.Lt = p.Lt; m.Ks = p.Ks; m.Kd = p.Kd; m.rx = p.rx; m.ry = p.ry; m.rz = p.rz;
    m.half_rho = 0.5 * rho;
    return m;
}

RtiConst make_rti_const(const kite_nmpc_config& c) {
    RtiConst r;
    std::memset(&r, 0, sizeof(r));
    r.N = c.N; r.M = c.M; r.K = c.qp_iters; r.n = 4 * c.N + 2;
    r.shift = c.shift;
    r.lo_fin = std::isfinite(c.lbx[0]) ? 1 : 0;
    r.hi_fin = std::isfinite(c.ubx[0]) ? 1 : 0;
    r.dt = c.dt; r.h = c.dt / c.M;
    for (int i = 0; i < 3; ++i) {
        r.sqQ_dt[i] = std::sqrt(c.dt * c.Q[i]);
        r.sqQ_T[i] = std::sqrt(c.Q[i]);
        r.Sr[i] = c.Sx[6 + i];
    }
    r.sw = std::sqrt(c.dt * c.W);
    r.sv = c.Sx[14];
    r.vref = c.vref;
    for (int j = 0; j < 4; ++j) {
        r.Rdiag[j] = c.dt * c.R[j] * c.Su[j] * c.Su[j];
        r.Rraw[j] = c.R[j];
        r.Su[j] = c.Su[j];
        r.lbu[j] = c.lbu[j]; r.ubu[j] = c.ubu[j];
    }
    r.Sx13 = c.Sx[13]; r.Sx14 = c.Sx[14];
    for (int i = 0; i < 15; ++i) { r.lbx[i] = c.lbx[i]; r.ubx[i] = c.ubx[i]; }
    r.flex = c.theta_flex;
    r.min_speed = c.min_speed;
    r.path_R = c.path_radius; r.path_alt = c.path_altitude;
    for (int i = 0; i < 4; ++i) r.pq[i] = c.path_q[i];
    r.path_K = c.path_harmonics;
    static_assert(KITE_PATH_NC == 2 * KITE_PATH_MAX_HARMONICS + 1, "path coefficient layout");
    for (int a = 0; a < 3; ++a)
        for (int j = 0; j < KITE_PATH_NC; ++j) r.pF[a][j] = c.path_harmonics ? c.path_fourier[a][j] : 0.0;
    r.delay = c.delay;
    r.delay_steps = c.delay_steps;
    r.delay_node = (int)std::lround(c.delay / c.dt);
    r.sens_fp32 = c.sens_fp32;
    return r;
}

// Constants of the multiple-shooting QP (qp_ric.inc; oracle build_msqp):
// per stage slot j (0..12 kite states, 13..15 T dE dR, 16 theta, 17 thetadot,
// 18 Uv) its bound and scale, and the inequality rows per stage type.
kite::RicConst make_ric_const(const kite_nmpc_config& c) {
    kite::RicConst r;
    std::memset(&r, 0, sizeof(r));
    r.soft_w = c.qp_soft_weight;
    r.lm = c.qp_lm;
    r.hth = c.dt * c.Sx[13] / c.Sx[14];
    r.g0 = 0.5 * c.dt * c.dt * c.Sx[13] / c.Su[3];
    r.g1 = c.dt * c.Sx[14] / c.Su[3];
    for (int a = 0; a < 3; ++a) {
        r.sq[0][a] = std::sqrt(c.dt * c.Q[a]);
        r.sq[1][a] = std::sqrt(c.Q[a]);
    }
    r.sw = std::sqrt(c.dt * c.W);
    r.ctheta = 1.0 / c.Sx[13];
    for (int q = 0; q < 4; ++q) r.Rh[q] = c.dt * c.R[q];
    for (int j = 0; j < 20; ++j) { r.lb[j] = -INFINITY; r.ub[j] = INFINITY; r.sc[j] = 1.0; }
    for (int i = 0; i < 13; ++i) { r.lb[i] = c.lbx[i]; r.ub[i] = c.ubx[i]; r.sc[i] = c.Sx[i]; }
    for (int q = 0; q < 4; ++q) {
        const int j = q < 3 ? 13 + q : 18;
        r.lb[j] = c.lbu[q]; r.ub[j] = c.ubu[q]; r.sc[j] = c.Su[q];
    }
    r.lb[16] = -c.theta_flex; r.ub[16] = c.theta_flex; r.sc[16] = c.Sx[13];
    r.lb[17] = -c.theta_flex; r.ub[17] = c.theta_flex; r.sc[17] = c.Sx[14];
    int nC = 0;
    for (int t = 0; t < 3; ++t) {
        int pairs = 0;
        r.lomask[t] = 0; r.himask[t] = 0;
        for (int j = 0; j < 20; ++j) {
            const bool state = j < 13, ctrl = (j >= 13 && j < 16) || j == 18, theta = (j == 16 || j == 17);
            const bool rows = (state && t > 0) || (ctrl && t < 2) || (theta && t == 0);
            if (!rows) continue;
            if (std::isfinite(r.lb[j])) { r.lomask[t] |= 1 << j; pairs += state ? 2 : 1; }
            if (std::isfinite(r.ub[j])) { r.himask[t] |= 1 << j; pairs += state ? 2 : 1; }
            if (std::isfinite(r.lb[j]) || std::isfinite(r.ub[j])) r.bslot[t][r.nb[t]++] = (int8_t)j;
        }
        nC += pairs * (t == 1 ? c.N - 1 : 1);
    }
    r.nC = nC;
    return r;
}

int validate_config(const kite_nmpc_config& c) {
    if (c.N < 1 || c.N > KITE_NMAX) return KITE_EINVAL;
    if (c.M < 1 || c.M > 64) return KITE_EINVAL;
    if (c.qp_iters < 0 || c.qp_iters > 200) return KITE_EINVAL;
    if (!(c.dt > 0.0) || !std::isfinite(c.dt)) return KITE_EINVAL;
    for (int i = 0; i < 15; ++i) if (!(c.Sx[i] != 0.0) || !std::isfinite(c.Sx[i])) return KITE_EINVAL;
    for (int i = 0; i < 4; ++i) {
        if (!(c.Su[i] != 0.0) || !std::isfinite(c.Su[i])) return KITE_EINVAL;
        if (!std::isfinite(c.lbu[i]) || !std::isfinite(c.ubu[i]) || !(c.lbu[i] < c.ubu[i])) return KITE_EINVAL;
    }
    // state bounds: ordered, no NaN; theta / thetadot (13, 14) are free in the
    // reference (nmpf_node.cpp:59-63) and not enforced here -- refuse finite ones
    // rather than drop them silently
    for (int i = 0; i < 15; ++i) if (!(c.lbx[i] <= c.ubx[i])) return KITE_EINVAL;
    for (int i = 13; i < 15; ++i)
        if (!(std::isinf(c.lbx[i]) && c.lbx[i] < 0.0 && std::isinf(c.ubx[i]) && c.ubx[i] > 0.0)) return KITE_EINVAL;
    for (int i = 0; i < 3; ++i) if (!(c.Q[i] >= 0.0)) return KITE_EINVAL;
    for (int i = 0; i < 4; ++i) if (!(c.R[i] >= 0.0)) return KITE_EINVAL;
    if (!(c.W >= 0.0) || !(c.theta_flex > 0.0)) return KITE_EINVAL;
    if (c.qp_kernel < 0 || c.qp_kernel > 3) return KITE_EINVAL;
    // the multiple-shooting QP's soft-row weight and LM term (the condensed
    // kernels 1 / 2 ignore both): soft_w > 2 z0 keeps the start point of
    // every soft row dual feasible (z2 = soft_w - z0 > z0, kite::RIC_Z0)
    const int qk = c.qp_kernel ? c.qp_kernel : (c.N == 20 ? 2 : 3);
    if (qk == 3) {
        if (!(c.qp_soft_weight > kite::RIC_SOFT_WEIGHT_MIN) || !std::isfinite(c.qp_soft_weight)) return KITE_EINVAL;
        if (!(c.qp_lm >= 0.0) || !std::isfinite(c.qp_lm)) return KITE_EINVAL;
    }
    if (c.sens_fp32 < 0 || c.sens_fp32 > 1) return KITE_EINVAL;
    if (!(c.delay >= 0.0) || !std::isfinite(c.delay) || std::lround(c.delay / c.dt) > c.N) return KITE_EINVAL;
    if (c.delay > 0.0 && (c.delay_steps < 1 || c.delay_steps > 64)) return KITE_EINVAL;
    if (c.path_harmonics < 0 || c.path_harmonics > KITE_PATH_MAX_HARMONICS) return KITE_EINVAL;
    for (int a = 0; a < 3; ++a)
        for (int j = 0; j < 2 * c.path_harmonics + 1; ++j)
            if (!std::isfinite(c.path_fourier[a][j])) return KITE_EINVAL;
    return KITE_OK;
}

int check_device(int dev) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return KITE_ENODEV;
    if (dev < 0 || dev >= count) return KITE_ENODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return KITE_ENODEV;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return KITE_ENODEV;
    return KITE_OK;
}

int ensure_scratch(kite_nmpc_ctx* ctx, size_t bytes) {
    if (bytes <= ctx->scratch_bytes) return KITE_OK;
    if (ctx->scratch) (void)hipFree(ctx->scratch);
    ctx->scratch = nullptr;
    ctx->scratch_bytes = 0;
    HIP_TRY(hipMalloc(&ctx->scratch, bytes));
    ctx->scratch_bytes = bytes;
    return KITE_OK;
}

void free_ctx(kite_nmpc_ctx* ctx) {
    double** bufs[] = {&ctx->X, &ctx->U, &ctx->x0, &ctx->AB, &ctx->DEF, &ctx->Hs, &ctx->hs,
                       &ctx->Cr, &ctx->cl, &ctx->cu, &ctx->hmax, &ctx->u0, &ctx->diag, &ctx->kkt,
                       &ctx->scratch, &ctx->Htl, &ctx->Hab, &ctx->Hbb, &ctx->wstep, &ctx->wind};
    for (double** p : bufs) if (*p) { (void)hipFree(*p); *p = nullptr; }
    if (ctx->dconst) { (void)hipFree(ctx->dconst); ctx->dconst = nullptr; }
    if (ctx->status) { (void)hipFree(ctx->status); ctx->status = nullptr; }
    if (ctx->iters) { (void)hipFree(ctx->iters); ctx->iters = nullptr; }
    if (ctx->order) { (void)hipFree(ctx->order); ctx->order = nullptr; }
    for (auto& e : ctx->ev) if (e) { (void)hipEventDestroy(e); e = nullptr; }
    for (auto& e : ctx->ring) if (e) (void)hipEventDestroy(e);
    ctx->ring.clear();
    for (auto& g : ctx->gexec) if (g) { (void)hipGraphExecDestroy(g); g = nullptr; }
    if (ctx->h_in) { (void)hipHostFree(ctx->h_in); ctx->h_in = nullptr; }
    if (ctx->h_out) { (void)hipHostFree(ctx->h_out); ctx->h_out = nullptr; }
    if (ctx->d_out) { (void)hipFree(ctx->d_out); ctx->d_out = nullptr; }
    if (ctx->own_stream) { (void)hipStreamDestroy(ctx->own_stream); ctx->own_stream = nullptr; }
}

// The multiple-shooting QP reads (rc, ricc) from device memory (ctx->dconst):
// re-uploaded on `s` when the host copy changed since the last upload.
int upload_dconst(kite_nmpc_ctx* ctx, hipStream_t s) {
    constexpr size_t roff = (sizeof(kite::RtiConst) + 255) / 256 * 256;
    static_assert(roff + sizeof(kite::RicConst) <= 4096, "dconst holds both constant blocks");
    unsigned char blob[roff + sizeof(kite::RicConst)] = {};
    std::memcpy(blob, &ctx->rc, sizeof(kite::RtiConst));
    std::memcpy(blob + roff, &ctx->ricc, sizeof(kite::RicConst));
    if (ctx->dconst_host.size() != sizeof(blob) || std::memcmp(ctx->dconst_host.data(), blob, sizeof(blob))) {
        // the host mirror is what the device holds: set only once the copy
        // is enqueued (a failed copy leaves it empty, so the next step retries)
        ctx->dconst_host.clear();
        ctx->dconst_stage.assign(blob, blob + sizeof(blob));
        HIP_TRY(hipMemcpyAsync(ctx->dconst, ctx->dconst_stage.data(), sizeof(blob), hipMemcpyHostToDevice, s));
        ctx->dconst_host.swap(ctx->dconst_stage);
    }
    return KITE_OK;
}

// Runs the RTI kernels on ctx->stream.  x0: B x 15 measured states in device
// memory (ctx->x0, or the caller's buffer for kite_nmpc_step_device: the
// prologue reads it in stream order, as a copy would).
int run_step(kite_nmpc_ctx* ctx, const double* x0) {
    hipStream_t s = ctx->stream;
    const int B = ctx->B;
    // events: the last-step set (cfg.timing) or the next slot of the ring
    hipEvent_t* ev = nullptr;
    if (ctx->ring_used < ctx->ring_cap && ctx->ring_phase++ % ctx->ring_stride == 0)
        ev = &ctx->ring[(size_t)ctx->ring_used++ * KITE_NEV];
    else if (ctx->cfg.timing)
        ev = ctx->ev;
    if (ev) HIP_TRY(hipEventRecord(ev[0], s));
    const double* wind = ctx->has_wind ? ctx->wind : nullptr;
    if (ctx->cold_dirty) HIP_TRY(hipMemsetAsync(ctx->order + 2 * B + 1, 0, sizeof(int32_t), s));
    ctx->cold_dirty = true;
    HIP_TRY(kite::launch_prologue(ctx->mc, ctx->rc, B, ctx->warm ? 1 : 0, x0, ctx->X, ctx->U, ctx->status,
                                  wind, ctx->order + 2 * B + 1, s));
    if (ev) HIP_TRY(hipEventRecord(ev[1], s));
    HIP_TRY(kite::launch_rk4_sens(ctx->mc, ctx->rc, B, ctx->X, ctx->U, ctx->AB, ctx->DEF, wind, s));
    if (ev) HIP_TRY(hipEventRecord(ev[2], s));
    if (!ctx->ric)
        HIP_TRY(kite::launch_condense(ctx->rc, B, ctx->X, ctx->U, ctx->AB, ctx->DEF, ctx->Hs, ctx->hs, ctx->Cr,
                                      ctx->cl, ctx->cu, ctx->hmax, ctx->tiled ? 1 : 0, ctx->Htl, ctx->Hab,
                                      ctx->Hbb, s));
    // QP dispatch order from the previous step's iteration counts (ctx->iters[0, B))
    HIP_TRY(kite::launch_qp_order(ctx->rc, B, ctx->iters, ctx->order, ctx->order + B, s));
    ctx->cold_dirty = false;
    if (ev) HIP_TRY(hipEventRecord(ev[3], s));
    if (ctx->ric) {
        constexpr size_t roff = (sizeof(kite::RtiConst) + 255) / 256 * 256;
        { const int urc = upload_dconst(ctx, s); if (urc) return urc; }
        const auto* Cd = reinterpret_cast<const kite::RtiConst*>(ctx->dconst);
        const auto* Rd = reinterpret_cast<const kite::RicConst*>(static_cast<const unsigned char*>(ctx->dconst) + roff);
        HIP_TRY(kite::launch_qp_ric(ctx->rc, ctx->ricc, Cd, Rd, B, ctx->AB, ctx->DEF, ctx->X, ctx->U, ctx->u0,
                                    ctx->diag, ctx->status, ctx->kkt, ctx->iters, ctx->iters + B, ctx->order,
                                    ctx->Hs, s, ev ? ev[5] : nullptr));
    }
    else if (ctx->tiled)
        HIP_TRY(kite::launch_qp_tiled(ctx->mc, ctx->rc, B, ctx->Htl, ctx->Hab, ctx->Hbb, ctx->hs, ctx->Cr, ctx->cl,
                                      ctx->cu, ctx->hmax, ctx->AB, ctx->DEF, ctx->X, ctx->U, ctx->u0, ctx->diag,
                                      ctx->status, ctx->kkt, ctx->iters, ctx->order, ctx->order + B, ctx->wstep,
                                      s, ev ? ev[5] : nullptr));
    else
        HIP_TRY(kite::launch_qp(ctx->mc, ctx->rc, B, ctx->Hs, ctx->hs, ctx->Cr, ctx->cl, ctx->cu, ctx->hmax, ctx->AB,
                                ctx->DEF, ctx->X, ctx->U, ctx->u0, ctx->diag, ctx->status, ctx->kkt, ctx->iters,
                                ctx->order, ctx->order + B, s, ev ? ev[5] : nullptr));
    if (ev) HIP_TRY(hipEventRecord(ev[4], s));
    ctx->timed_step = (ev == ctx->ev);
    ctx->warm = true;
    return KITE_OK;
}

// ---- the captured host step (kite_nmpc_step) -------------------------------
// output staging layout in bytes: u0 B x 4 | traj B x (N+1) x 15 | ctrl B x N x 4 |
// diag B x 6 (doubles) | status B (int32)
struct OutLayout {
    size_t u0, traj, ctrl, diag, status, total;
};
OutLayout out_layout(size_t B, size_t N) {
    OutLayout o;
    o.u0 = 0;
    o.traj = o.u0 + B * 4 * sizeof(double);
    o.ctrl = o.traj + B * (N + 1) * 15 * sizeof(double);
    o.diag = o.ctrl + B * N * 4 * sizeof(double);
    o.status = o.diag + B * 6 * sizeof(double);
    o.total = o.status + B * sizeof(int32_t);
    return o;
}

int ensure_staging(kite_nmpc_ctx* ctx) {
    if (ctx->h_in && ctx->h_out && ctx->d_out) return KITE_OK;
    const OutLayout o = out_layout(ctx->B, ctx->cfg.N);
    if (!ctx->h_in) HIP_TRY(hipHostMalloc((void**)&ctx->h_in, (size_t)ctx->B * 15 * sizeof(double)));
    if (!ctx->h_out) HIP_TRY(hipHostMalloc((void**)&ctx->h_out, o.total));
    if (!ctx->d_out) HIP_TRY(hipMalloc((void**)&ctx->d_out, o.total));
    return KITE_OK;
}

// Captures x0 in (pinned -> device), run_step and the outputs out (one fused
// publish kernel into device staging, one copy to pinned memory) for the given
// warm flag.  No events are recorded (the caller checks that no timing is on).
int capture_step(kite_nmpc_ctx* ctx, int warm) {
    const size_t B = ctx->B, N = ctx->cfg.N;
    const OutLayout o = out_layout(B, N);
    hipStream_t cs = ctx->own_stream;
    hipStream_t saved_stream = ctx->stream;
    const bool saved_warm = ctx->warm;
    ctx->stream = cs;
    ctx->warm = warm != 0;
    HIP_TRY(hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed));
    int rc = KITE_OK;
    hipError_t e = hipMemcpyAsync(ctx->x0, ctx->h_in, B * 15 * sizeof(double), hipMemcpyHostToDevice, cs);
    if (e == hipSuccess) rc = run_step(ctx, ctx->x0);
    if (e == hipSuccess && rc == KITE_OK)
        e = kite::launch_publish((int)B, (int)N, ctx->u0, ctx->X, ctx->U, ctx->diag, ctx->status,
                                 (double*)(ctx->d_out + o.u0), (double*)(ctx->d_out + o.traj),
                                 (double*)(ctx->d_out + o.ctrl), (double*)(ctx->d_out + o.diag),
                                 (int32_t*)(ctx->d_out + o.status), cs);
    if (e == hipSuccess && rc == KITE_OK) e = hipMemcpyAsync(ctx->h_out, ctx->d_out, o.total, hipMemcpyDeviceToHost, cs);
    hipGraph_t graph = nullptr;
    const hipError_t ee = hipStreamEndCapture(cs, &graph);
    ctx->stream = saved_stream;
    ctx->warm = saved_warm;
    if (rc != KITE_OK || e != hipSuccess || ee != hipSuccess) {
        if (graph) (void)hipGraphDestroy(graph);
        return rc != KITE_OK ? rc : hip_fail(e != hipSuccess ? e : ee);
    }
    hipGraphExec_t ex = nullptr;
    e = hipGraphInstantiate(&ex, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (e != hipSuccess) return hip_fail(e);
    if (ctx->gexec[warm]) (void)hipGraphExecDestroy(ctx->gexec[warm]);
    ctx->gexec[warm] = ex;
    ctx->gexec_gen[warm] = ctx->graph_gen;
    return KITE_OK;
}

// ---- minimal YAML reader for the two-level kite parameter file -----------
std::string trim(const std::string& s) {
    size_t a = 0, b = s.size();
    while (a < b && std::isspace((unsigned char)s[a])) ++a;
    while (b > a && std::isspace((unsigned char)s[b - 1])) --b;
    return s.substr(a, b - a);
}

}  // namespace

extern "C" {

int kite_nmpc_api_version(void) { return KITE_NMPC_API_VERSION; }

const char* kite_nmpc_strerror(int code) {
    switch (code) {
        case KITE_OK: return "ok";
        case KITE_EINVAL: return "invalid argument";
        case KITE_EHIP: return "HIP runtime error";
        case KITE_ENOMEM: return "out of memory";
        case KITE_ENODEV: return "no usable gfx950 device";
        case KITE_EIO: return "cannot read parameter file";
        case KITE_EPARSE: return "parameter file: missing key or bad number";
        case KITE_ESTATE: return "call not valid in this state";
        default: return "unknown error";
    }
}

int kite_params_load_yaml(const char* path, kite_params* out) {
    if (!path || !out) return KITE_EINVAL;
    std::ifstream f(path);
    if (!f) return KITE_EIO;
    std::map<std::string, double> kv;
    std::string line, section;
    while (std::getline(f, line)) {
        const size_t hash = line.find('#');
        if (hash != std::string::npos) line = line.substr(0, hash);
        if (trim(line).empty()) continue;
        const bool indented = std::isspace((unsigned char)line[0]);
        const size_t colon = line.find(':');
        if (colon == std::string::npos) return KITE_EPARSE;
        const std::string key = trim(line.substr(0, colon));
        const std::string val = trim(line.substr(colon + 1));
        if (!indented) {
            section = val.empty() ? key : std::string();
            continue;
        }
        if (section.empty()) return KITE_EPARSE;
        char* end = nullptr;
        const double d = std::strtod(val.c_str(), &end);
        if (val.empty() || end == val.c_str() || *end != '\0') return KITE_EPARSE;
        kv[section + "." + key] = d;
    }
    struct Field { const char* key; double* dst; bool required; };
    kite_params p;
    std::memset(&p, 0, sizeof(p));
    const Field fields[] = {
        {"geometry.b", &p.b, true}, {"geometry.c", &p.c, true}, {"geometry.AR", &p.AR, true},
        {"geometry.S", &p.S, true}, {"geometry.lam", &p.lam, true}, {"geometry.St", &p.St, true},
        {"geometry.lt", &p.lt, true}, {"geometry.Sf", &p.Sf, true}, {"geometry.lf", &p.lf, true},
        {"geometry.Xac", &p.Xac, true},
        {"inertia.mass", &p.mass, true}, {"inertia.Ixx", &p.Ixx, true}, {"inertia.Iyy", &p.Iyy, true},
        {"inertia.Izz", &p.Izz, true}, {"inertia.Ixz", &p.Ixz, true},
        {"aerodynamic.CL0", &p.CL0, true}, {"aerodynamic.CL0_tail", &p.CL0_tail, true},
        {"aerodynamic.CLa_total", &p.CLa_total, true}, {"aerodynamic.CLa_wing", &p.CLa_wing, true},
        {"aerodynamic.CLa_tail", &p.CLa_tail, true}, {"aerodynamic.e_oswald", &p.e_oswald, true},
        {"aerodynamic.CD0_total", &p.CD0_total, true}, {"aerodynamic.CD0_wing", &p.CD0_wing, true},
        {"aerodynamic.CD0_tail", &p.CD0_tail, true}, {"aerodynamic.CYb", &p.CYb, true},
        {"aerodynamic.CYb_vtail", &p.CYb_vtail, true}, {"aerodynamic.Cm0", &p.Cm0, true},
        {"aerodynamic.Cma", &p.Cma, true}, {"aerodynamic.Cn0", &p.Cn0, true}, {"aerodynamic.Cnb", &p.Cnb, true},
        {"aerodynamic.Cl0", &p.Cl0, true}, {"aerodynamic.Clb", &p.Clb, true}, {"aerodynamic.CLq", &p.CLq, true},
        {"aerodynamic.Cmq", &p.Cmq, true}, {"aerodynamic.CYr", &p.CYr, true}, {"aerodynamic.Cnr", &p.Cnr, true},
        {"aerodynamic.Clr", &p.Clr, true}, {"aerodynamic.CYp", &p.CYp, true}, {"aerodynamic.Clp", &p.Clp, true},
        {"aerodynamic.Cnp", &p.Cnp, true}, {"aerodynamic.CLde", &p.CLde, true},
        {"aerodynamic.CYdr", &p.CYdr, true}, {"aerodynamic.Cmde", &p.Cmde, true},
        {"aerodynamic.Cndr", &p.Cndr, true}, {"aerodynamic.Cldr", &p.Cldr, true},
        {"aerodynamic.CDde", &p.CDde, true},
        {"tether.length", &p.Lt, true}, {"tether.Ks", &p.Ks, true}, {"tether.Kd", &p.Kd, true},
        {"tether.rx", &p.rx, false}, {"tether.ry", &p.ry, false}, {"tether.rz", &p.rz, false},
    };
    for (const Field& fd : fields) {
        auto it = kv.find(fd.key);
        if (it == kv.end()) {
            if (fd.required) return KITE_EPARSE;
            *fd.dst = 0.0;
        } else {
            *fd.dst = it->second;
        }
    }
    *out = p;
    return KITE_OK;
}

void kite_nmpc_default_config(kite_nmpc_config* c) {
    if (!c) return;
    std::memset(c, 0, sizeof(*c));
    const double inf = INFINITY, pi = M_PI;
    c->N = 20; c->M = 2; c->qp_iters = 16; c->shift = 1; c->device = 0; c->timing = 0;
    c->delay = 0.0; c->delay_steps = 16;
    c->sens_fp32 = 0;
    c->dt = 0.05;
    const double Q[3] = {1e3, 1e3, 1e4};
    const double R[4] = {1e-4, 1e-1, 1e-1, 1e-3};
    std::memcpy(c->Q, Q, sizeof(Q));
    std::memcpy(c->R, R, sizeof(R));
    c->W = 1e-3;
    const double Sx[15] = {0.1, 1 / 3.0, 1 / 3.0, 1 / 2.0, 1 / 5.0, 1 / 2.0, 1 / 3.0, 1 / 3.0, 1 / 3.0,
                           1.0, 1.0, 1.0, 1.0, 1 / 6.28, 1 / 6.28};
    const double Su[4] = {1 / 0.15, 1 / 0.2618, 1 / 0.2618, 1 / 5.0};
    std::memcpy(c->Sx, Sx, sizeof(Sx));
    std::memcpy(c->Su, Su, sizeof(Su));
    const double lbx[15] = {2.0, -inf, -inf, -4 * pi, -4 * pi, -4 * pi, -inf, -inf, -inf,
                            -1.01, -1.01, -1.01, -1.01, -inf, -inf};
    const double ubx[15] = {inf, inf, inf, 4 * pi, 4 * pi, 4 * pi, inf, inf, inf,
                            1.01, 1.01, 1.01, 1.01, inf, inf};
    std::memcpy(c->lbx, lbx, sizeof(lbx));
    std::memcpy(c->ubx, ubx, sizeof(ubx));
    const double sat = 7.0 * pi / 180.0;
    const double lbu[4] = {0.1, -sat, -sat, -5.0};
    const double ubu[4] = {0.15, sat, sat, 5.0};
    std::memcpy(c->lbu, lbu, sizeof(lbu));
    std::memcpy(c->ubu, ubu, sizeof(ubu));
    c->vref = 4.0;
    c->path_radius = 2.65;
    c->path_altitude = 0.0;
    c->path_q[0] = std::cos(pi / 8); c->path_q[1] = 0.0; c->path_q[2] = std::sin(pi / 8); c->path_q[3] = 0.0;
    c->theta_flex = 0.78;
    c->min_speed = 2.1;
    c->qp_soft_weight = 1e3;
    c->qp_lm = 10.0;
}

int kite_nmpc_create(const kite_params* params, const kite_nmpc_config* cfg, int32_t batch,
                     kite_nmpc_ctx** out) {
    if (!params || !cfg || !out || batch < 1) return KITE_EINVAL;
    *out = nullptr;
    int rc = validate_config(*cfg);
    if (rc) return rc;
    rc = check_device(cfg->device);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(cfg->device));
    kite_nmpc_ctx* ctx = new kite_nmpc_ctx();
    ctx->params = *params;
    ctx->cfg = *cfg;
    ctx->B = batch;
    ctx->device = cfg->device;
    ctx->mc = make_model_const(*params);
    ctx->rc = make_rti_const(*cfg);
    const size_t B = (size_t)batch, N = (size_t)cfg->N, n = 4 * N + 2;
    const bool tiled_ok = kite::qp_tiled_supported(ctx->rc);
    if (cfg->qp_kernel == 2 && !tiled_ok) { delete ctx; return KITE_EINVAL; }
    // auto: the register-tiled condensed QP at N == 20 (fastest there, well
    // conditioned over a 1 s horizon), the multiple-shooting QP otherwise
    const int qk = cfg->qp_kernel != 0 ? cfg->qp_kernel : (cfg->N == 20 ? 2 : 3);
    ctx->ric = qk == 3;
    ctx->tiled = qk == 2;
    if (ctx->ric) {
        ctx->ricc = make_ric_const(*cfg);
        if (kite::qp_ric_lds_bytes(ctx->rc, ctx->ricc) > 160 * 1024 - 1024) { delete ctx; return KITE_EINVAL; }
    }
    const size_t na = 4 * N;
    const size_t ntile = (N / 4) * (N / 4 + 1) / 2;
    struct Alloc { double** p; size_t count; };
    const Alloc allocs[] = {
        {&ctx->X, B * (N + 1) * 15}, {&ctx->U, B * N * 4}, {&ctx->x0, B * 15},
        {&ctx->AB, B * N * 13 * 16}, {&ctx->DEF, B * N * 13},
        // ric: Hs is k_qp_ric's workspace (the factor rows S_k, qp_ric_ws_doubles per kite)
        {&ctx->Hs, ctx->tiled ? 1 : (ctx->ric ? B * kite::qp_ric_ws_doubles(ctx->rc) : B * n * n)}, {&ctx->hs, ctx->ric ? 1 : B * n},
        {&ctx->Cr, ctx->ric ? 1 : B * N * n}, {&ctx->cl, ctx->ric ? 1 : B * N}, {&ctx->cu, ctx->ric ? 1 : B * N},
        {&ctx->hmax, B}, {&ctx->u0, B * 4}, {&ctx->diag, B * 6}, {&ctx->kkt, B},
        {&ctx->Htl, ctx->tiled ? B * ntile * 256 : 1}, {&ctx->Hab, ctx->tiled ? B * na * 2 : 1},
        {&ctx->Hbb, ctx->tiled ? B * 4 : 1}, {&ctx->wstep, ctx->tiled ? 2 * B * n : 1},
    };
    for (const Alloc& a : allocs) {
        if (hipMalloc(a.p, a.count * sizeof(double)) != hipSuccess) { free_ctx(ctx); delete ctx; return KITE_ENOMEM; }
        (void)hipMemset(*a.p, 0, a.count * sizeof(double));
    }
    if (hipMalloc(&ctx->status, B * sizeof(int32_t)) != hipSuccess ||
        hipMalloc(&ctx->iters, 4 * B * sizeof(int32_t)) != hipSuccess ||
        hipMalloc(&ctx->order, (3 * (size_t)B + 2) * sizeof(int32_t)) != hipSuccess ||
        hipMalloc(&ctx->dconst, 4096) != hipSuccess) { free_ctx(ctx); delete ctx; return KITE_ENOMEM; }
    (void)hipMemset(ctx->status, 0, B * sizeof(int32_t));
    (void)hipMemset(ctx->order, 0, (3 * (size_t)B + 2) * sizeof(int32_t));
    // [0, B): QP iterations of the last step; running sums since timing_start:
    // [B, 2B) QP iterations, [2B, 3B) steps ending outside the state box (status
    // bit 8), [3B, 4B) (node, state) pairs outside it (kite_nmpc_state_bound_stats)
    (void)hipMemset(ctx->iters, 0, 4 * B * sizeof(int32_t));
    if (hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking) != hipSuccess) {
        free_ctx(ctx); delete ctx; return KITE_EHIP;
    }
    ctx->stream = ctx->own_stream;
    {
        const char* ng = std::getenv("KITE_NMPC_NO_GRAPH");
        ctx->graph_off = ng && ng[0] == '1';
    }
    for (auto& e : ctx->ev)
        if (hipEventCreateWithFlags(&e, kTimingEventFlags) != hipSuccess) { free_ctx(ctx); delete ctx; return KITE_EHIP; }
    if (hipDeviceSynchronize() != hipSuccess) { free_ctx(ctx); delete ctx; return KITE_EHIP; }
    *out = ctx;
    return KITE_OK;
}

void kite_nmpc_destroy(kite_nmpc_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    free_ctx(ctx);
    delete ctx;
}

int kite_nmpc_batch(const kite_nmpc_ctx* ctx) { return ctx ? ctx->B : KITE_EINVAL; }

int kite_nmpc_set_bounds(kite_nmpc_ctx* ctx, const double* lbx15, const double* ubx15, const double* lbu4,
                         const double* ubu4) {
    if (!ctx) return KITE_EINVAL;
    kite_nmpc_config c = ctx->cfg;
    if (lbx15) std::memcpy(c.lbx, lbx15, sizeof(c.lbx));
    if (ubx15) std::memcpy(c.ubx, ubx15, sizeof(c.ubx));
    if (lbu4) std::memcpy(c.lbu, lbu4, sizeof(c.lbu));
    if (ubu4) std::memcpy(c.ubu, ubu4, sizeof(c.ubu));
    const int rc = validate_config(c);
    if (rc) return rc;
    ctx->cfg = c;
    ctx->rc = make_rti_const(c);
    if (ctx->ric) ctx->ricc = make_ric_const(c);     // the QP's bounds
    ++ctx->graph_gen;                                // captured kernels hold rc by value
    return KITE_OK;
}

int kite_nmpc_set_reference_velocity(kite_nmpc_ctx* ctx, double vref) {
    if (!ctx || !std::isfinite(vref)) return KITE_EINVAL;
    ctx->cfg.vref = vref;
    ctx->rc = make_rti_const(ctx->cfg);
    ++ctx->graph_gen;
    return KITE_OK;
}

int kite_nmpc_reset(kite_nmpc_ctx* ctx) {
    if (!ctx) return KITE_EINVAL;
    ctx->warm = false;
    return KITE_OK;
}

int kite_nmpc_set_wind(kite_nmpc_ctx* ctx, const double* wind) {
    if (!ctx) return KITE_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));      // the wind buffer lives on the context's device
    bool any = false;
    if (wind) {
        for (size_t e = 0; e < (size_t)ctx->B * 3; ++e) {
            if (!std::isfinite(wind[e])) return KITE_EINVAL;
            any = any || wind[e] != 0.0;
        }
    }
    ++ctx->graph_gen;                                    // the wind selects other kernels
    if (!any) { ctx->has_wind = false; return KITE_OK; }   // the reference model
    if (!ctx->wind) HIP_TRY(hipMalloc(&ctx->wind, (size_t)ctx->B * 3 * sizeof(double)));
    // ordered with the steps on the context stream (the host array may be
    // reused as soon as this returns: synchronous on that stream)
    HIP_TRY(hipMemcpyAsync(ctx->wind, wind, (size_t)ctx->B * 3 * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    ctx->has_wind = true;
    return KITE_OK;
}

int kite_nmpc_set_stream(kite_nmpc_ctx* ctx, void* hip_stream) {
    if (!ctx) return KITE_EINVAL;
    ctx->stream = (hipStream_t)hip_stream;
    return KITE_OK;
}

int kite_nmpc_use_own_stream(kite_nmpc_ctx* ctx) {
    if (!ctx) return KITE_EINVAL;
    ctx->stream = ctx->own_stream;
    return KITE_OK;
}

int kite_nmpc_synchronize(kite_nmpc_ctx* ctx) {
    if (!ctx) return KITE_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return KITE_OK;
}

int kite_nmpc_step_device(kite_nmpc_ctx* ctx, const double* d_x0, double* d_u0, double* d_traj, double* d_ctrl,
                          double* d_diag, int32_t* d_status) {
    if (!ctx || !d_x0) return KITE_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    const size_t B = ctx->B, N = ctx->cfg.N;
    hipStream_t s = ctx->stream;
    int rc = run_step(ctx, d_x0);
    if (rc) return rc;
    HIP_TRY(kite::launch_publish((int)B, (int)N, ctx->u0, ctx->X, ctx->U, ctx->diag, ctx->status, d_u0, d_traj,
                                 d_ctrl, d_diag, d_status, s));
    return KITE_OK;
}

int kite_nmpc_step(kite_nmpc_ctx* ctx, const double* x0, double* u0_out, double* traj_out, double* ctrl_out,
                   kite_mpc_diagnostic* diag_out, int32_t* status_out) {
    if (!ctx || !x0) return KITE_EINVAL;
    const auto t0 = std::chrono::steady_clock::now();
    HIP_TRY(hipSetDevice(ctx->device));
    const size_t B = ctx->B, N = ctx->cfg.N;
    hipStream_t s = ctx->stream;
    // the captured step: no per-kernel timing requested (cfg.timing, a live
    // timing_start ring); otherwise the launches below record their events
    if (!ctx->graph_off && !ctx->cfg.timing && ctx->ring_used >= ctx->ring_cap) {
        int rc = ensure_staging(ctx);
        if (rc) return rc;
        if (ctx->ric) { rc = upload_dconst(ctx, s); if (rc) return rc; }   // outside the graph
        const int w = ctx->warm ? 1 : 0;
        if (!ctx->gexec[w] || ctx->gexec_gen[w] != ctx->graph_gen) {
            rc = capture_step(ctx, w);
            if (rc) return rc;
        }
        std::memcpy(ctx->h_in, x0, B * 15 * sizeof(double));
        HIP_TRY(hipGraphLaunch(ctx->gexec[w], s));
        HIP_TRY(hipStreamSynchronize(s));
        ctx->warm = true;
        ctx->timed_step = false;
        const OutLayout o = out_layout(B, N);
        if (u0_out) std::memcpy(u0_out, ctx->h_out + o.u0, B * 4 * sizeof(double));
        if (traj_out) std::memcpy(traj_out, ctx->h_out + o.traj, B * (N + 1) * 15 * sizeof(double));
        if (ctrl_out) std::memcpy(ctrl_out, ctx->h_out + o.ctrl, B * N * 4 * sizeof(double));
        if (status_out) std::memcpy(status_out, ctx->h_out + o.status, B * sizeof(int32_t));
        if (diag_out) {
            static_assert(sizeof(kite_mpc_diagnostic) == 6 * sizeof(double), "diagnostic layout");
            std::memcpy(diag_out, ctx->h_out + o.diag, B * 6 * sizeof(double));
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            for (size_t b = 0; b < B; ++b) diag_out[b].comp_time_ms = ms;
        }
        return KITE_OK;
    }
    HIP_TRY(hipMemcpyAsync(ctx->x0, x0, B * 15 * sizeof(double), hipMemcpyHostToDevice, s));
    int rc = run_step(ctx, ctx->x0);
    if (rc) return rc;
    if (u0_out) HIP_TRY(hipMemcpyAsync(u0_out, ctx->u0, B * 4 * sizeof(double), hipMemcpyDeviceToHost, s));
    if (traj_out) HIP_TRY(hipMemcpyAsync(traj_out, ctx->X, B * (N + 1) * 15 * sizeof(double), hipMemcpyDeviceToHost, s));
    if (ctrl_out) HIP_TRY(hipMemcpyAsync(ctrl_out, ctx->U, B * N * 4 * sizeof(double), hipMemcpyDeviceToHost, s));
    if (diag_out) {
        static_assert(sizeof(kite_mpc_diagnostic) == 6 * sizeof(double), "diagnostic layout");
        HIP_TRY(hipMemcpyAsync(diag_out, ctx->diag, B * 6 * sizeof(double), hipMemcpyDeviceToHost, s));
    }
    if (status_out) HIP_TRY(hipMemcpyAsync(status_out, ctx->status, B * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (diag_out) {
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        for (size_t b = 0; b < B; ++b) diag_out[b].comp_time_ms = ms;
    }
    return KITE_OK;
}

int kite_nmpc_get_solution(kite_nmpc_ctx* ctx, double* traj, double* ctrl) {
    if (!ctx) return KITE_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    const size_t B = ctx->B, N = ctx->cfg.N;
    if (traj) HIP_TRY(hipMemcpyAsync(traj, ctx->X, B * (N + 1) * 15 * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    if (ctrl) HIP_TRY(hipMemcpyAsync(ctrl, ctx->U, B * N * 4 * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return KITE_OK;
}

int kite_nmpc_set_solution(kite_nmpc_ctx* ctx, const double* traj, const double* ctrl) {
    if (!ctx || !traj || !ctrl) return KITE_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    const size_t B = ctx->B, N = ctx->cfg.N;
    HIP_TRY(hipMemcpyAsync(ctx->X, traj, B * (N + 1) * 15 * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(ctx->U, ctrl, B * N * 4 * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    // non-finite plans are flagged like a NaN iterate: the next step restarts them cold
    std::vector<int32_t> st(B, 0);
    for (size_t b = 0; b < B; ++b) {
        bool fin = true;
        for (size_t e = 0; e < (N + 1) * 15; ++e) fin &= std::isfinite(traj[b * (N + 1) * 15 + e]);
        for (size_t e = 0; e < N * 4; ++e) fin &= std::isfinite(ctrl[b * N * 4 + e]);
        st[b] = fin ? 0 : KITE_ST_NAN;
    }
    HIP_TRY(hipMemcpyAsync(ctx->status, st.data(), B * sizeof(int32_t), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    ctx->warm = true;
    return KITE_OK;
}

// ---- model-level entry points: host in/out, scratch on device -------------
extern "C++" {
namespace {
template <class Launch>
int run_items(kite_nmpc_ctx* ctx, const std::vector<std::pair<const double*, size_t>>& in,
              const std::vector<std::pair<double*, size_t>>& out, Launch launch) {
    HIP_TRY(hipSetDevice(ctx->device));
    size_t total = 0;
    for (auto& p : in) total += p.second;
    for (auto& p : out) total += p.second;
    int rc = ensure_scratch(ctx, total * sizeof(double));
    if (rc) return rc;
    std::vector<double*> din, dout;
    double* cur = ctx->scratch;
    hipStream_t s = ctx->stream;
    for (auto& p : in) {
        din.push_back(cur);
        if (p.first) HIP_TRY(hipMemcpyAsync(cur, p.first, p.second * sizeof(double), hipMemcpyHostToDevice, s));
        cur += p.second;
    }
    for (auto& p : out) { dout.push_back(cur); cur += p.second; }
    HIP_TRY(launch(din, dout, s));
    for (size_t i = 0; i < out.size(); ++i)
        if (out[i].first)
            HIP_TRY(hipMemcpyAsync(out[i].first, dout[i], out[i].second * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return KITE_OK;
}
}  // namespace
}  // extern "C++"

int kite_nmpc_dynamics(kite_nmpc_ctx* ctx, int32_t count, const double* x15, const double* u4, double* f15) {
    if (!ctx || count < 1 || !x15 || !u4 || !f15) return KITE_EINVAL;
    const size_t c = count;
    return run_items(ctx, {{x15, c * 15}, {u4, c * 4}}, {{f15, c * 15}},
                     [&](std::vector<double*>& i, std::vector<double*>& o, hipStream_t s) {
                         return kite::launch_dynamics(ctx->mc, count, i[0], i[1], o[0], s);
                     });
}

int kite_nmpc_jacobian(kite_nmpc_ctx* ctx, int32_t count, const double* x13, const double* u3, double* Jx,
                       double* Ju) {
    if (!ctx || count < 1 || !x13 || !u3 || !Jx || !Ju) return KITE_EINVAL;
    const size_t c = count;
    return run_items(ctx, {{x13, c * 13}, {u3, c * 3}}, {{Jx, c * 169}, {Ju, c * 39}},
                     [&](std::vector<double*>& i, std::vector<double*>& o, hipStream_t s) {
                         return kite::launch_jacobian(ctx->mc, count, i[0], i[1], o[0], o[1], s);
                     });
}

int kite_nmpc_predict(kite_nmpc_ctx* ctx, int32_t count, const double* x15, const double* u4, double tf,
                      int32_t steps, double* x15_out) {
    if (!ctx || count < 1 || !x15 || !u4 || !x15_out || steps < 1 || !std::isfinite(tf)) return KITE_EINVAL;
    const size_t c = count;
    const double h = tf / steps;
    return run_items(ctx, {{x15, c * 15}, {u4, c * 4}}, {{x15_out, c * 15}},
                     [&](std::vector<double*>& i, std::vector<double*>& o, hipStream_t s) {
                         return kite::launch_predict(ctx->mc, count, i[0], i[1], h, steps, o[0], s);
                     });
}

// ---- Chebyshev collocation evaluator (chebyshev.hpp) ------------------------
extern "C++" {
namespace {
// CGL differentiation matrix of degree n on x_j = cos(j pi / n) (chebyshev.hpp:130-153)
std::vector<double> cheb_D(int n) {
    const int m = n + 1;
    std::vector<double> x(m), c(m), D((size_t)m * m);
    for (int j = 0; j < m; ++j) {
        x[j] = std::cos(j * (M_PI / n));
        c[j] = ((j == 0 || j == n) ? 2.0 : 1.0) * ((j % 2) ? -1.0 : 1.0);
    }
    for (int i = 0; i < m; ++i) {       // Dn = c (1/c)' / (dX + I);  D = Dn - diag(rowsum(Dn))
        double row = 0.0;
        for (int j = 0; j < m; ++j) {
            const double v = (c[i] / c[j]) / (x[i] - x[j] + (i == j ? 1.0 : 0.0));
            D[(size_t)i * m + j] = v;
            row += v;
        }
        D[(size_t)i * m + i] -= row;
    }
    return D;
}
// Clenshaw-Curtis weights on the CGL points (chebyshev.hpp:156-195)
std::vector<double> cheb_weights(int n) {
    std::vector<double> w(n + 1, 0.0), v(std::max(0, n - 1), 1.0);
    auto th = [&](int j) { return j * (M_PI / n); };
    if (n % 2 == 0) {
        w[0] = w[n] = 1.0 / ((double)n * n - 1.0);
        for (int k = 1; k <= n / 2 - 1; ++k)
            for (int i = 0; i < n - 1; ++i) v[i] -= 2.0 * std::cos(2.0 * k * th(i + 1)) / (4.0 * k * k - 1.0);
        for (int i = 0; i < n - 1; ++i) v[i] -= std::cos(n * th(i + 1)) / ((double)n * n - 1.0);
    } else {
        w[0] = w[n] = 1.0 / ((double)n * n);
        for (int k = 1; k <= (n - 1) / 2; ++k)
            for (int i = 0; i < n - 1; ++i) v[i] -= 2.0 * std::cos(2.0 * k * th(i + 1)) / (4.0 * k * k - 1.0);
    }
    for (int i = 0; i < n - 1; ++i) w[i + 1] = 2.0 * v[i] / n;
    return w;
}
}  // namespace
}  // extern "C++"

void kite_colloc_default_config(kite_colloc_config* c) {
    if (!c) return;
    std::memset(c, 0, sizeof(*c));
    kite_nmpc_config n;
    kite_nmpc_default_config(&n);
    c->poly_order = 5; c->num_segments = 2; c->use_R = 1;       // kiteNMPF.cpp:82-83
    c->t0 = 0.0; c->tf = 1.0;                                    // kiteNMPF.cpp:88
    for (int i = 0; i < 3; ++i) c->Q[i] = n.Q[i];
    for (int i = 0; i < 4; ++i) { c->R[i] = n.R[i]; c->Su[i] = n.Su[i]; }
    c->W = n.W;
    for (int i = 0; i < 15; ++i) c->Sx[i] = n.Sx[i];
    c->vref = n.Sx[14] * n.vref;                                 // setReferenceVelocity (kiteNMPF.h:34)
    c->mayer_scale = 1.0;
    c->path_radius = n.path_radius; c->path_altitude = n.path_altitude;
    for (int i = 0; i < 4; ++i) c->path_q[i] = n.path_q[i];
    c->path_harmonics = n.path_harmonics;
    std::memcpy(c->path_fourier, n.path_fourier, sizeof(c->path_fourier));
}

int kite_nmpc_colloc_eval(kite_nmpc_ctx* ctx, const kite_colloc_config* cfg, int32_t count, const double* z,
                          double* G, double* J, double* jac) {
    if (!ctx || !cfg || count < 1 || !z || !G || !J) return KITE_EINVAL;
    const int P = cfg->poly_order, S = cfg->num_segments, n = P * S + 1;
    if (P < 1 || S < 1 || n > 32 || !(cfg->tf > cfg->t0)) return KITE_EINVAL;
    for (int i = 0; i < 15; ++i) if (!(cfg->Sx[i] != 0.0) || !std::isfinite(cfg->Sx[i])) return KITE_EINVAL;
    for (int i = 0; i < 4; ++i) if (!(cfg->Su[i] != 0.0) || !std::isfinite(cfg->Su[i])) return KITE_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    // composite differentiation matrix (chebyshev.hpp:198-232) and node weights
    const std::vector<double> D = cheb_D(P), w = cheb_weights(P);
    std::vector<double> tab((size_t)n * n + n, 0.0);
    if (S < 2) {
        for (int i = 0; i <= P; ++i) for (int j = 0; j <= P; ++j) tab[(size_t)i * n + j] = D[(size_t)i * (P + 1) + j];
    } else {
        for (int i = 0; i <= P; ++i)
            for (int j = 0; j <= P; ++j) tab[(size_t)(n - P - 1 + i) * n + (n - P - 1 + j)] = D[(size_t)i * (P + 1) + j];
        for (int k = 0; k < (S - 1) * P; k += P)
            for (int i = 0; i < P; ++i)
                for (int j = 0; j <= P; ++j) tab[(size_t)(k + i) * n + (k + j)] = D[(size_t)i * (P + 1) + j];
    }
    kite::CollocConst C;
    std::memset(&C, 0, sizeof(C));
    C.nodes = n; C.use_R = cfg->use_R;
    C.t_scale = (cfg->tf - cfg->t0) / (2.0 * S);
    C.mayer_scale = cfg->mayer_scale;
    for (int k = 0; k < S; ++k)                                  // chebyshev.hpp:303-322
        for (int m = 0; m <= P; ++m) tab[(size_t)n * n + k * P + m] += C.t_scale * w[m];
    for (int i = 0; i < 3; ++i) C.Q[i] = cfg->Q[i];
    for (int i = 0; i < 4; ++i) { C.R[i] = cfg->R[i]; C.Su[i] = cfg->Su[i]; C.iSu[i] = 1.0 / cfg->Su[i]; }
    for (int i = 0; i < 15; ++i) { C.Sx[i] = cfg->Sx[i]; C.iSx[i] = 1.0 / cfg->Sx[i]; }
    C.W = cfg->W; C.vref = cfg->vref;
    C.path_R = cfg->path_radius; C.path_alt = cfg->path_altitude;
    for (int i = 0; i < 4; ++i) C.pq[i] = cfg->path_q[i];
    if (cfg->path_harmonics < 0 || cfg->path_harmonics > KITE_PATH_MAX_HARMONICS) return KITE_EINVAL;
    C.path_K = cfg->path_harmonics;
    for (int a = 0; a < 3; ++a)
        for (int j = 0; j < KITE_PATH_NC; ++j) C.pF[a][j] = cfg->path_harmonics ? cfg->path_fourier[a][j] : 0.0;

    const size_t c = count, nz = (size_t)n * 19, ng = (size_t)n * 15, nj = jac ? c * n * 15 * 19 : 0;
    int rc = ensure_scratch(ctx, (tab.size() + c * nz + c * ng + c + nj) * sizeof(double));
    if (rc) return rc;
    double *dtab = ctx->scratch, *dz = dtab + tab.size(), *dG = dz + c * nz, *dJ = dG + c * ng, *djac = dJ + c;
    hipStream_t s = ctx->stream;
    HIP_TRY(hipMemcpyAsync(dtab, tab.data(), tab.size() * sizeof(double), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(dz, z, c * nz * sizeof(double), hipMemcpyHostToDevice, s));
    HIP_TRY(kite::launch_colloc(ctx->mc, C, count, dtab, dz, dG, dJ, jac ? djac : nullptr, s));
    HIP_TRY(hipMemcpyAsync(G, dG, c * ng * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(J, dJ, c * sizeof(double), hipMemcpyDeviceToHost, s));
    if (jac) HIP_TRY(hipMemcpyAsync(jac, djac, nj * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return KITE_OK;
}

// ---- extended Kalman filter (kiteEKF.cpp) ----------------------------------
void kite_ekf_default_covariances(double* W169, double* V49, double* P0_169) {
    // kiteEKF.cpp:6-13: W = diag(S_v, S_w, S_r, S_q)^2, V = diag(...)^2; P0 = 10 W (:26)
    const double sd_w[13] = {0.5, 0.5, 0.5, 0.5, 0.5, 0.5, 0.5, 0.1, 0.1, 0.01, 0.05, 0.05, 0.05};
    const double sd_v[7] = {0.01, 0.01, 0.01, 0.0001, 0.005, 0.005, 0.005};
    for (int i = 0; i < 169; ++i) {
        if (W169) W169[i] = 0.0;
        if (P0_169) P0_169[i] = 0.0;
    }
    for (int i = 0; i < 13; ++i) {
        if (W169) W169[i * 13 + i] = sd_w[i] * sd_w[i];
        if (P0_169) P0_169[i * 13 + i] = 10.0 * (sd_w[i] * sd_w[i]);
    }
    if (V49) {
        for (int i = 0; i < 49; ++i) V49[i] = 0.0;
        for (int i = 0; i < 7; ++i) V49[i * 7 + i] = sd_v[i] * sd_v[i];
    }
}

int kite_nmpc_ekf_step_device(kite_nmpc_ctx* ctx, int32_t count, double dt, double* d_x13, const double* d_u3,
                              double* d_P169, const double* d_z7, const double* d_W169, const double* d_V49) {
    if (!ctx || count < 1 || !d_x13 || !d_u3 || !d_P169 || !d_W169 || (d_z7 && !d_V49) || !std::isfinite(dt))
        return KITE_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(kite::launch_ekf(ctx->mc, count, dt, d_x13, d_u3, d_P169, d_z7, d_W169, d_V49, ctx->stream));
    return KITE_OK;
}

int kite_nmpc_ekf_step(kite_nmpc_ctx* ctx, int32_t count, double dt, double* x13, const double* u3, double* P169,
                       const double* z7, const double* W169, const double* V49) {
    if (!ctx || count < 1 || !x13 || !u3 || !P169 || !W169 || (z7 && !V49) || !std::isfinite(dt)) return KITE_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    const size_t c = count;
    const size_t nx = c * 13, nu = c * 3, np = c * 169, nz = z7 ? c * 7 : 0;
    int rc = ensure_scratch(ctx, (nx + nu + np + nz + 169 + 49) * sizeof(double));
    if (rc) return rc;
    double *dx = ctx->scratch, *du = dx + nx, *dP = du + nu, *dz = dP + np, *dW = dz + nz, *dV = dW + 169;
    hipStream_t s = ctx->stream;
    HIP_TRY(hipMemcpyAsync(dx, x13, nx * sizeof(double), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(du, u3, nu * sizeof(double), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(dP, P169, np * sizeof(double), hipMemcpyHostToDevice, s));
    if (z7) HIP_TRY(hipMemcpyAsync(dz, z7, nz * sizeof(double), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(dW, W169, 169 * sizeof(double), hipMemcpyHostToDevice, s));
    if (V49) HIP_TRY(hipMemcpyAsync(dV, V49, 49 * sizeof(double), hipMemcpyHostToDevice, s));
    HIP_TRY(kite::launch_ekf(ctx->mc, count, dt, dx, du, dP, z7 ? dz : nullptr, dW, dV, s));
    HIP_TRY(hipMemcpyAsync(x13, dx, nx * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(P169, dP, np * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return KITE_OK;
}

int kite_nmpc_rk4_sens(kite_nmpc_ctx* ctx, int32_t count, const double* x15, const double* u4, double tf,
                       int32_t M, double* xnext, double* A, double* Bm) {
    if (!ctx || count < 1 || !x15 || !u4 || !xnext || !A || !Bm || M < 1 || !std::isfinite(tf)) return KITE_EINVAL;
    const size_t c = count;
    const double h = tf / M;
    // scratch outputs (no host copy): X2 [c][2][15], AB [c][13][16], DEF [c][13]
    return run_items(ctx, {{x15, c * 15}, {u4, c * 4}},
                     {{xnext, c * 15}, {A, c * 225}, {Bm, c * 60}, {nullptr, c * 30}, {nullptr, c * 208},
                      {nullptr, c * 13}},
                     [&](std::vector<double*>& i, std::vector<double*>& o, hipStream_t s) {
                         return kite::launch_rk4_sens_items(ctx->mc, ctx->rc.sens_fp32, count, M, h, i[0], i[1],
                                                            o[0], o[1], o[2], o[3], o[4], o[5], s);
                     });
}

int kite_nmpc_closest_point(kite_nmpc_ctx* ctx, int32_t count, const double* pos, const double* guess,
                            double* theta_out) {
    if (!ctx || count < 1 || !pos || !theta_out) return KITE_EINVAL;
    const size_t c = count;
    std::vector<double> g;
    if (!guess) g.assign(c, 0.0);
    return run_items(ctx, {{pos, c * 3}, {guess ? guess : g.data(), c}}, {{theta_out, c}},
                     [&](std::vector<double*>& i, std::vector<double*>& o, hipStream_t s) {
                         return kite::launch_closest_point(ctx->rc, count, i[0], i[1], o[0], s);
                     });
}

int kite_nmpc_path_eval(const kite_nmpc_config* cfg, int32_t count, const double* theta, double* P3, double* dP3) {
    if (!cfg || count < 0 || (count > 0 && (!theta || !P3))) return KITE_EINVAL;
    // rotation by the unit quaternion (w, u): v' = (w^2 - u.u) v + 2 (u.v) u - 2 w (u x v)
    // (q^-1 (x) [0, v] (x) q, the sandwich of nmpf_node.cpp:35-39)
    const double w = cfg->path_q[0], ux = cfg->path_q[1], uy = cfg->path_q[2], uz = cfg->path_q[3];
    const double ww_uu = w * w - (ux * ux + uy * uy + uz * uz);
    auto rot = [&](double vx, double vy, double vz, double* out) {
        const double ud = ux * vx + uy * vy + uz * vz;
        const double cx = uy * vz - uz * vy, cy = uz * vx - ux * vz, cz = ux * vy - uy * vx;
        out[0] = ww_uu * vx + 2.0 * ud * ux - 2.0 * w * cx;
        out[1] = ww_uu * vy + 2.0 * ud * uy - 2.0 * w * cy;
        out[2] = ww_uu * vz + 2.0 * ud * uz - 2.0 * w * cz;
    };
    if (cfg->path_harmonics < 0 || cfg->path_harmonics > KITE_PATH_MAX_HARMONICS) return KITE_EINVAL;
    for (int32_t i = 0; i < count; ++i) {
        const double s = std::sin(theta[i]), c = std::cos(theta[i]);
        double p[3], dp[3];
        kite::path_curve(cfg->path_harmonics, cfg->path_radius, cfg->path_altitude, cfg->path_fourier, c, s, p, dp);
        rot(p[0], p[1], p[2], P3 + 3 * (size_t)i);
        if (dP3) rot(dp[0], dp[1], dp[2], dP3 + 3 * (size_t)i);
    }
    return KITE_OK;
}

int kite_nmpc_kernel_times(kite_nmpc_ctx* ctx, double* ms, int32_t n) {
    if (!ctx || !ms || n < 1) return KITE_EINVAL;
    if (!ctx->timed_step) return KITE_ESTATE;
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipEventSynchronize(ctx->ev[4]));
    float v[6];
    for (int i = 0; i < 4; ++i) HIP_TRY(hipEventElapsedTime(&v[i], ctx->ev[i], ctx->ev[i + 1]));
    HIP_TRY(hipEventElapsedTime(&v[4], ctx->ev[0], ctx->ev[4]));
    HIP_TRY(hipEventElapsedTime(&v[5], ctx->ev[3], ctx->ev[5]));
    const int m = n < 6 ? n : 6;
    for (int i = 0; i < m; ++i) ms[i] = v[i];
    return m;
}

int kite_nmpc_timing_start(kite_nmpc_ctx* ctx, int32_t max_steps) {
    return kite_nmpc_timing_start_sampled(ctx, max_steps, 1);
}

int kite_nmpc_timing_start_sampled(kite_nmpc_ctx* ctx, int32_t max_steps, int32_t stride) {
    if (!ctx || max_steps < 0 || stride < 1) return KITE_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    const size_t need = (size_t)max_steps * KITE_NEV;
    while (ctx->ring.size() < need) {
        hipEvent_t e;
        HIP_TRY(hipEventCreateWithFlags(&e, kTimingEventFlags));
        ctx->ring.push_back(e);
    }
    ctx->ring_cap = max_steps;
    ctx->ring_used = 0;
    ctx->ring_stride = stride;
    ctx->ring_phase = 0;
    // restart the per-instance running sums (ctx->iters[B, 4B))
    HIP_TRY(hipMemsetAsync(ctx->iters + ctx->B, 0, 3 * (size_t)ctx->B * sizeof(int32_t), ctx->stream));
    return KITE_OK;
}

int kite_nmpc_timing_read(kite_nmpc_ctx* ctx, double* sums_ms, int32_t n) {
    if (!ctx || !sums_ms || n < 1) return KITE_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    double acc[6] = {0, 0, 0, 0, 0, 0};
    const int used = ctx->ring_used;
    if (used > 0) HIP_TRY(hipEventSynchronize(ctx->ring[(size_t)(used - 1) * KITE_NEV + 4]));
    for (int i = 0; i < used; ++i) {
        hipEvent_t* ev = &ctx->ring[(size_t)i * KITE_NEV];
        float v;
        for (int k = 0; k < 4; ++k) {
            HIP_TRY(hipEventElapsedTime(&v, ev[k], ev[k + 1]));
            acc[k] += v;
        }
        HIP_TRY(hipEventElapsedTime(&v, ev[0], ev[4]));
        acc[4] += v;
        HIP_TRY(hipEventElapsedTime(&v, ev[3], ev[5]));
        acc[5] += v;
    }
    const int m = n < 6 ? n : 6;
    for (int i = 0; i < m; ++i) sums_ms[i] = acc[i];
    ctx->ring_cap = 0;
    ctx->ring_used = 0;
    return used;
}

int kite_nmpc_qp_stats(kite_nmpc_ctx* ctx, double* kkt, int32_t* iters) {
    if (!ctx) return KITE_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    const size_t B = ctx->B;
    if (kkt) HIP_TRY(hipMemcpyAsync(kkt, ctx->kkt, B * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    if (iters) HIP_TRY(hipMemcpyAsync(iters, ctx->iters, B * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return KITE_OK;
}

int kite_nmpc_qp_iteration_sum(kite_nmpc_ctx* ctx, int64_t* sum) {
    if (!ctx || !sum) return KITE_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    std::vector<int32_t> acc(ctx->B);
    HIP_TRY(hipMemcpyAsync(acc.data(), ctx->iters + ctx->B, acc.size() * sizeof(int32_t), hipMemcpyDeviceToHost,
                           ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    int64_t t = 0;
    for (int32_t v : acc) t += v;
    *sum = t;
    return KITE_OK;
}

int kite_nmpc_state_bound_stats(kite_nmpc_ctx* ctx, int64_t* steps_outside, int64_t* rows_outside) {
    if (!ctx) return KITE_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    std::vector<int32_t> acc(2 * (size_t)ctx->B);
    HIP_TRY(hipMemcpyAsync(acc.data(), ctx->iters + 2 * ctx->B, acc.size() * sizeof(int32_t), hipMemcpyDeviceToHost,
                           ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    int64_t a = 0, r = 0;
    for (int i = 0; i < ctx->B; ++i) { a += acc[i]; r += acc[(size_t)ctx->B + i]; }
    if (steps_outside) *steps_outside = a;
    if (rows_outside) *rows_outside = r;
    return KITE_OK;
}

int kite_nmpc_get_qp(kite_nmpc_ctx* ctx, int32_t instance, double* H, double* h, double* C, double* cl,
                     double* cu) {
    if (!ctx || instance < 0 || instance >= ctx->B) return KITE_EINVAL;
    if (ctx->ric) return KITE_ESTATE;      // the multiple-shooting QP is never condensed
    HIP_TRY(hipSetDevice(ctx->device));
    const size_t N = ctx->cfg.N, n = 4 * N + 2, b = instance;
    hipStream_t s = ctx->stream;
    if (H && !ctx->tiled)
        HIP_TRY(hipMemcpyAsync(H, ctx->Hs + b * n * n, n * n * sizeof(double), hipMemcpyDeviceToHost, s));
    if (H && ctx->tiled) {
        // reassemble the full matrix from the C-layout tiles (lane l: column l&15,
        // rows (l>>4) + 4r), H_ab and H_bb
        const size_t na = 4 * N, nt = N / 4, ntile = nt * (nt + 1) / 2;
        std::vector<double> tl(ntile * 256), ab(na * 2), bb(4);
        HIP_TRY(hipMemcpyAsync(tl.data(), ctx->Htl + b * ntile * 256, tl.size() * sizeof(double), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(ab.data(), ctx->Hab + b * na * 2, ab.size() * sizeof(double), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(bb.data(), ctx->Hbb + b * 4, 4 * sizeof(double), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        int t = 0;
        for (int I = 0; I < (int)nt; ++I)
            for (int J = 0; J <= I; ++J, ++t)
                for (int r = 0; r < 4; ++r)
                    for (int l = 0; l < 64; ++l) {
                        const size_t gi = 16 * I + (l >> 4) + 4 * r, gj = 16 * J + (l & 15);
                        const double v = tl[(size_t)t * 256 + r * 64 + l];
                        H[gi * n + gj] = v;
                        H[gj * n + gi] = v;
                    }
        for (size_t i = 0; i < na; ++i)
            for (size_t c = 0; c < 2; ++c) { H[i * n + na + c] = ab[i * 2 + c]; H[(na + c) * n + i] = ab[i * 2 + c]; }
        for (size_t c = 0; c < 2; ++c)
            for (size_t d = 0; d < 2; ++d) H[(na + c) * n + na + d] = bb[c * 2 + d];
    }
    if (h) HIP_TRY(hipMemcpyAsync(h, ctx->hs + b * n, n * sizeof(double), hipMemcpyDeviceToHost, s));
    if (C) HIP_TRY(hipMemcpyAsync(C, ctx->Cr + b * N * n, N * n * sizeof(double), hipMemcpyDeviceToHost, s));
    if (cl) HIP_TRY(hipMemcpyAsync(cl, ctx->cl + b * N, N * sizeof(double), hipMemcpyDeviceToHost, s));
    if (cu) HIP_TRY(hipMemcpyAsync(cu, ctx->cu + b * N, N * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return KITE_OK;
}

}  // extern "C"
