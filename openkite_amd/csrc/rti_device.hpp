// rti_device.hpp -- device helpers shared by the RTI kernels (rti_kernels.hip)
// and the multiple-shooting QP (ric_kernels.hip): cross-lane primitives of one
// 64-wide wavefront, NaN-propagating reductions, the path, pivot safeguards.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "kite_model.hpp"
#include "rti_kernels.hpp"

namespace kite {

typedef double double4v __attribute__((ext_vector_type(4)));

// Compiler barriers written as inline asm always hold one real instruction
// (asm volatile("s_nop 0" ...)): the hazard recognizer counts each inline-asm
// statement as one wait state, so an empty one can shorten a required VALU ->
// DPP / readlane / MFMA gap by one and read a stale register.

// ---------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------
// a wave-uniform double moved to SGPRs (frees two VGPRs for as long as it lives)
__device__ __forceinline__ double uniform_d(double v) {
    const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
    const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readlane_d(double v, int lane) {
    int lo = __double2loint(v), hi = __double2hiint(v);
    lo = __builtin_amdgcn_readlane(lo, lane);
    hi = __builtin_amdgcn_readlane(hi, lane);
    return __hiloint2double(hi, lo);
}
// LDS exchange between the lanes of ONE wavefront: a wavefront-scope fence
// pair around the wave barrier (no s_barrier; used where a block is a single
// wave, or where one wave of a block works alone)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// ---------------------------------------------------------------------------
// cross-lane primitives, all VALU (no LDS round trip).  Lane semantics of the
// gfx950 permlane swaps, probed on the device (tools/probes/lane_ops.hip):
//   permlane16_swap(x, x) -> {rows [0,0,2,2], rows [1,1,3,3]}   (16-lane rows)
//   permlane32_swap(x, x) -> {lanes [0-31, 0-31], lanes [32-63, 32-63]}
//   DPP row_newbcast:p    -> lane p of each 16-lane row, to the whole row
// All of these must be called in wave-uniform control flow.
// ---------------------------------------------------------------------------
// 64-bit DPP move.  Every control used here (row_ror, row_newbcast, quad_perm)
// reads an in-row lane, so the old value is dead: bound_ctrl with no old
// operand lets the compiler skip the zero-initialisation of the destination,
// and row_newbcast becomes a single v_mov_b64_dpp.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const long x = __builtin_amdgcn_update_dpp((long)0, __builtin_bit_cast(long, v), CTRL, 0xF, 0xF, true);
    return __builtin_bit_cast(double, x);
}
// {value of rows [0,0,2,2], value of rows [1,1,3,3]}
__device__ __forceinline__ void swap16_d(double v, double& ev, double& od) {
    const auto L = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
    const auto H = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
    ev = __hiloint2double((int)H[0], (int)L[0]);
    od = __hiloint2double((int)H[1], (int)L[1]);
}
// {value of lanes [0-31, 0-31], value of lanes [32-63, 32-63]}
__device__ __forceinline__ void swap32_d(double v, double& lo_half, double& hi_half) {
    const auto L = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
    const auto H = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
    lo_half = __hiloint2double((int)H[0], (int)L[0]);
    hi_half = __hiloint2double((int)H[1], (int)L[1]);
}
// reduce over the 16 lanes of each row (every lane gets its row's result)
template <class Op>
__device__ __forceinline__ double row_reduce16(double v, Op op) {
    v = op(v, dpp_d<0x128>(v));   // row_ror:8
    v = op(v, dpp_d<0x124>(v));   // row_ror:4
    v = op(v, dpp_d<0x122>(v));   // row_ror:2
    v = op(v, dpp_d<0x121>(v));   // row_ror:1
    return v;
}
// reduce over the 4 lanes l, l^16, l^32, l^48 (same position in each row)
template <class Op>
__device__ __forceinline__ double col_reduce4(double v, Op op) {
    double a, b;
    swap16_d(v, a, b);
    v = op(a, b);
    swap32_d(v, a, b);
    return op(a, b);
}
// value of row-group q (lanes 16q..16q+15), delivered to the same position of every row
__device__ __forceinline__ double bcast_rowgroup(double v, int q) {
    double a, b;
    swap16_d(v, a, b);
    const double t = (q & 1) ? b : a;
    swap32_d(t, a, b);
    return (q & 2) ? b : a;
}
struct OpAdd { __device__ double operator()(double a, double b) const { return a + b; } };
struct OpMax { __device__ double operator()(double a, double b) const { return fmax(a, b); } };
struct OpMin { __device__ double operator()(double a, double b) const { return fmin(a, b); } };
// RTI step safeguard threshold on the final QP residual (oracle QP_STEP_ACCEPT)
constexpr double QP_STEP_ACCEPT = 1e-6;

// NaN-propagating max (fmax drops NaN: a poisoned KKT residual must never
// read as converged)
__device__ __forceinline__ double nmax(double a, double b) { return (a != a || b != b) ? NAN : fmax(a, b); }
struct OpNMax { __device__ double operator()(double a, double b) const { return nmax(a, b); } };

__device__ __forceinline__ double row_sum16(double v) { return row_reduce16(v, OpAdd()); }
// four row sums at once (transpose-reduce): v[q] -> sum of v[q] over the 16
// lanes of each row, every lane.  Each butterfly level halves the values a lane
// carries (xor 8: keep the pair of bit 3; xor 7 (row_half_mirror): keep one by
// bit 2; xor 3, xor 1 (quad_perm): plain), so lane j ends with sum q = j >> 2,
// broadcast back by row_newbcast: 10 DPP moves + 5 adds + 6 selects instead of
// 4 x (8 DPP moves + 4 adds).  Every lane gets bitwise the same sums.
// `hi8` / `hi4`: bit 3 / bit 2 of the lane's position in its row.
__device__ __forceinline__ void row_sum16x4(double v[4], bool hi8, bool hi4) {
    const double k0 = hi8 ? v[2] : v[0], k1 = hi8 ? v[3] : v[1];
    const double s0 = hi8 ? v[0] : v[2], s1 = hi8 ? v[1] : v[3];
    const double a0 = k0 + dpp_d<0x128>(s0);           // row_ror:8 = xor 8
    const double a1 = k1 + dpp_d<0x128>(s1);
    const double kb = hi4 ? a1 : a0, sb = hi4 ? a0 : a1;
    double b = kb + dpp_d<0x141>(sb);                   // row_half_mirror = xor 7
    b += dpp_d<0x1B>(b);                                // quad_perm [3,2,1,0] = xor 3
    b += dpp_d<0xB1>(b);                                // quad_perm [1,0,3,2] = xor 1
    v[0] = dpp_d<0x150>(b);                             // row_newbcast: lane 4q holds sum q
    v[1] = dpp_d<0x154>(b);
    v[2] = dpp_d<0x158>(b);
    v[3] = dpp_d<0x15C>(b);
}
__device__ __forceinline__ double col_sum4(double v) { return col_reduce4(v, OpAdd()); }
__device__ __forceinline__ double wave_sum(double v) { return col_reduce4(row_reduce16(v, OpAdd()), OpAdd()); }
__device__ __forceinline__ double wave_max(double v) { return col_reduce4(row_reduce16(v, OpMax()), OpMax()); }
__device__ __forceinline__ double wave_nmax(double v) { return col_reduce4(row_reduce16(v, OpNMax()), OpNMax()); }
__device__ __forceinline__ double wave_min(double v) { return col_reduce4(row_reduce16(v, OpMin()), OpMin()); }
__device__ __forceinline__ int wave_or(int v) {
    // flags are 0/1: reuse the fp64 max path
    return wave_max((double)v) != 0.0 ? 1 : 0;
}

// Path P(theta) = q_r^-1 (x) [0, p(theta)] (x) q_r and dP/dtheta
// (nmpf_node.cpp:30-40; p: the circle or the Fourier curve, kite_path.hpp).
__device__ __forceinline__ void path_eval(const RtiConst& C, double th, double P[3], double dP[3]) {
    double s, c;
    sincos(th, &s, &c);
    double pc[3], dpc[3];
    path_curve(C.path_K, C.path_R, C.path_alt, C.pF, c, s, pc, dpc);
    const double qw = C.pq[0];
    const V3<double> qu{C.pq[1], C.pq[2], C.pq[3]};
    const double ww_uu = qw * qw - dot3(qu, qu);
    V3<double> p = rot_body(qw, qu, ww_uu, V3<double>{pc[0], pc[1], pc[2]});
    V3<double> dp = rot_body(qw, qu, ww_uu, V3<double>{dpc[0], dpc[1], dpc[2]});
    P[0] = p.x; P[1] = p.y; P[2] = p.z;
    dP[0] = dp.x; dP[1] = dp.y; dP[2] = dp.z;
}

// state-bound tolerance (oracle bound_tol)
__device__ __forceinline__ double bound_tol(double b) { return 1e-8 * fmax(1.0, fabs(b)); }

// Cholesky pivot safeguard (Wright 1999, see oracle/kite_oracle.cpp chol): a
// pivot <= 0 from rounding near convergence is replaced by a huge value,
// freezing that direction for the step; NaN stays NaN.
constexpr double KITE_PIV_BIG = 1e128;
__device__ __forceinline__ double piv_fix(double s) { return s <= 0.0 ? KITE_PIV_BIG : s; }
// 1/sqrt(p): v_rsq_f64 estimate y (~2^-23) + one third-order correction
// y (1 + e/2 + 3e^2/8), e = 1 - p y^2 (~1 ulp; the IEEE sqrt + division
// sequence is ~20 instructions)
__device__ __forceinline__ double fast_rsq(double p) {
    const double y = __builtin_amdgcn_rsq(p);
    const double e = fma(-p, y * y, 1.0);
    return fma(y * e, fma(e, 0.375, 0.5), y);
}

}  // namespace kite
