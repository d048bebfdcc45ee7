// kite_model.hpp -- device-side 6-DOF tethered kite ODE for gfx950.
//
// Same equations as KiteDynamics (src/kite_model/kite.cpp:197-317), written for
// the GPU:
//   * quaternion sandwich products q^-1 (x) v (x) q are evaluated with the
//     closed-form identity (w^2 - u.u) v + 2(u.v) u -/+ 2w (u x v) (exact for
//     non-unit q too, which the reference relies on: kite.cpp:317 keeps |q|
//     only approximately 1);
//   * the wind-frame rotations use cos/sin of the full angles obtained
//     algebraically (cos a = (v0+1e-4)/rho, sin b = v1/(V+1e-4)) instead of
//     four half-angle sincos calls; the coefficient formulas still use the
//     angles themselves (asin / atan2) exactly as kite.cpp:200-201;
//   * the scalar type is a template: double for the primal, Dual (value +
//     one tangent) for the Jacobian kernels, Dual2 / DualF2 (value + two
//     tangents, fp64 / fp32) for the forward sensitivities of k_rk4_sens2.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

namespace kite {

constexpr int NX = 15, NU = 4, NK = 13, NKU = 3;

// Model constants, precomputed on the host from kite_params (kite.cpp:93-175).
struct ModelConst {
    double inv_mass;
    double S, b, c;
    double CL0, CLa, CD0, inv_pieAR;            // CD = CD0 + (CL0+CLa a)^2 / (pi e AR)
    double kLq;                                  // 0.25 CLq c S rho
    double CYb, CYdr, kSF;                       // b rho S * 0.25
    double CYr, CYp;
    double CLde;
    double Cl0, Clb, Cldr, Clr, Clp, kRoll;      // 0.25 rho b^2 S
    double Cm0, Cma, Cmde, Cmq, kPitch;          // 0.25 S c^2 rho
    double Cn0, Cnb, Cndr, Cnp, Cnr, kYaw;       // 0.25 S b^2 rho
    double Ixx, Iyy, Izz, Ixz, Ji00, Ji02, Ji11, Ji22;   // J^-1 entries
    double Lt, Ks, Kd, rx, ry, rz;
    double half_rho;
};

constexpr double kGravity = 9.80665;  // kite.cpp:93
constexpr double kRho = 1.2985;       // kite.cpp:94

// ---------------------------------------------------------------------------
// Dual number: value + one directional derivative.
// ---------------------------------------------------------------------------
struct Dual {
    double v, t;
    Dual() = default;
    __host__ __device__ constexpr Dual(double a) : v(a), t(0.0) {}
    __host__ __device__ constexpr Dual(double a, double b) : v(a), t(b) {}
};
__device__ __forceinline__ Dual mk(double v, double t) { return Dual(v, t); }
__device__ __forceinline__ Dual operator+(Dual a, Dual b) { return mk(a.v + b.v, a.t + b.t); }
__device__ __forceinline__ Dual operator-(Dual a, Dual b) { return mk(a.v - b.v, a.t - b.t); }
__device__ __forceinline__ Dual operator-(Dual a) { return mk(-a.v, -a.t); }
__device__ __forceinline__ Dual operator*(Dual a, Dual b) { return mk(a.v * b.v, fma(a.t, b.v, a.v * b.t)); }
__device__ __forceinline__ Dual operator+(Dual a, double b) { return mk(a.v + b, a.t); }
__device__ __forceinline__ Dual operator+(double b, Dual a) { return mk(a.v + b, a.t); }
__device__ __forceinline__ Dual operator-(Dual a, double b) { return mk(a.v - b, a.t); }
__device__ __forceinline__ Dual operator-(double b, Dual a) { return mk(b - a.v, -a.t); }
__device__ __forceinline__ Dual operator*(Dual a, double b) { return mk(a.v * b, a.t * b); }
__device__ __forceinline__ Dual operator*(double b, Dual a) { return mk(a.v * b, a.t * b); }
// 1/d for the sensitivity kernel: v_rcp_f64 estimate r (~2^-23) and one
// third-order correction r (1 + e + e^2), e = 1 - d r -- ~1 ulp in 4
// instructions instead of the ~10 of the IEEE division sequence (the primal
// double path keeps IEEE division)
__device__ __forceinline__ double fast_rcp(double d) {
    const double r = __builtin_amdgcn_rcp(d);
    const double e = fma(-d, r, 1.0);
    return fma(r, fma(e, e, e), r);
}
// (the tangent formulas are written exactly as Dual2's, fma included, so that
// the one-tangent sensitivity kernel k_rk4_sens1 reproduces k_rk4_sens2 bit for bit)
__device__ __forceinline__ Dual operator/(Dual a, Dual b) {
    double ib = fast_rcp(b.v);
    double q = a.v * ib;
    return mk(q, fma(-q, b.t, a.t) * ib);
}
__device__ __forceinline__ Dual operator/(Dual a, double b) { double ib = fast_rcp(b); return mk(a.v * ib, a.t * ib); }
__device__ __forceinline__ Dual rcp(Dual a) { const double r = fast_rcp(a.v), nr2 = -r * r; return mk(r, a.t * nr2); }
__device__ __forceinline__ double rcp(double a) { return 1.0 / a; }

__device__ __forceinline__ double val(double a) { return a; }
__device__ __forceinline__ double val(Dual a) { return a.v; }

// sqrt with a caller-known reciprocal reuse
__device__ __forceinline__ double dsqrt(double a) { return sqrt(a); }
__device__ __forceinline__ Dual dsqrt(Dual a) { double s = sqrt(a.v); return mk(s, a.t * (0.5 * fast_rcp(s))); }
__device__ __forceinline__ double dexp(double a) { return exp(a); }
__device__ __forceinline__ Dual dexp(Dual a) { double e = exp(a.v); return mk(e, a.t * e); }
// asin(x) when sqrt(1-x^2) (= cos of the result) is already known
__device__ __forceinline__ double dasin(double x, double /*cosv*/) { return asin(x); }
__device__ __forceinline__ Dual dasin(Dual x, Dual cosv) { return mk(asin(x.v), x.t * fast_rcp(cosv.v)); }
// atan2(y,x) when x^2+y^2 is already known
__device__ __forceinline__ double datan2(double y, double x, double /*r2*/) { return atan2(y, x); }
__device__ __forceinline__ Dual datan2(Dual y, Dual x, Dual r2) {
    const double ir = fast_rcp(r2.v);
    return mk(atan2(y.v, x.v), fma(x.v, y.t, -(y.v * x.t)) * ir);
}

// ---------------------------------------------------------------------------
// Dual2: value + TWO directional derivatives (k_rk4_sens, fp64): the primal
// -- including its transcendentals -- is evaluated once for two tangent
// directions, so 8 lanes instead of 16 cover the 16 directions of a
// (kite, interval).
// ---------------------------------------------------------------------------
struct Dual2 {
    double v, a, b;
    Dual2() = default;
    __host__ __device__ constexpr Dual2(double x) : v(x), a(0.0), b(0.0) {}
    __host__ __device__ constexpr Dual2(double x, double ta, double tb) : v(x), a(ta), b(tb) {}
};
__device__ __forceinline__ Dual2 mk2(double v, double a, double b) { return Dual2(v, a, b); }
__device__ __forceinline__ Dual2 operator+(Dual2 x, Dual2 y) { return mk2(x.v + y.v, x.a + y.a, x.b + y.b); }
__device__ __forceinline__ Dual2 operator-(Dual2 x, Dual2 y) { return mk2(x.v - y.v, x.a - y.a, x.b - y.b); }
__device__ __forceinline__ Dual2 operator-(Dual2 x) { return mk2(-x.v, -x.a, -x.b); }
__device__ __forceinline__ Dual2 operator*(Dual2 x, Dual2 y) {
    return mk2(x.v * y.v, fma(x.a, y.v, x.v * y.a), fma(x.b, y.v, x.v * y.b));
}
__device__ __forceinline__ Dual2 operator+(Dual2 x, double c) { return mk2(x.v + c, x.a, x.b); }
__device__ __forceinline__ Dual2 operator+(double c, Dual2 x) { return mk2(x.v + c, x.a, x.b); }
__device__ __forceinline__ Dual2 operator-(Dual2 x, double c) { return mk2(x.v - c, x.a, x.b); }
__device__ __forceinline__ Dual2 operator-(double c, Dual2 x) { return mk2(c - x.v, -x.a, -x.b); }
__device__ __forceinline__ Dual2 operator*(Dual2 x, double c) { return mk2(x.v * c, x.a * c, x.b * c); }
__device__ __forceinline__ Dual2 operator*(double c, Dual2 x) { return mk2(x.v * c, x.a * c, x.b * c); }
__device__ __forceinline__ Dual2 operator/(Dual2 x, Dual2 y) {
    const double iy = fast_rcp(y.v);
    const double q = x.v * iy;
    return mk2(q, fma(-q, y.a, x.a) * iy, fma(-q, y.b, x.b) * iy);
}
__device__ __forceinline__ Dual2 operator/(Dual2 x, double c) {
    const double ic = fast_rcp(c);
    return mk2(x.v * ic, x.a * ic, x.b * ic);
}
__device__ __forceinline__ Dual2 rcp(Dual2 x) {
    const double r = fast_rcp(x.v), nr2 = -r * r;
    return mk2(r, x.a * nr2, x.b * nr2);
}
__device__ __forceinline__ double val(Dual2 x) { return x.v; }
__device__ __forceinline__ Dual2 dsqrt(Dual2 x) {
    const double s = sqrt(x.v), h = 0.5 * fast_rcp(s);
    return mk2(s, x.a * h, x.b * h);
}
__device__ __forceinline__ Dual2 dexp(Dual2 x) { const double e = exp(x.v); return mk2(e, x.a * e, x.b * e); }
__device__ __forceinline__ Dual2 dasin(Dual2 x, Dual2 cosv) {
    const double ic = fast_rcp(cosv.v);
    return mk2(asin(x.v), x.a * ic, x.b * ic);
}
__device__ __forceinline__ Dual2 datan2(Dual2 y, Dual2 x, Dual2 r2) {
    const double ir = fast_rcp(r2.v);
    return mk2(atan2(y.v, x.v), fma(x.v, y.a, -(y.v * x.a)) * ir, fma(x.v, y.b, -(y.v * x.b)) * ir);
}

// two fp32 tangents (mixed precision, config sens_fp32 = 1, k_rk4_sens2<DualF2>),
// packed: the tangent pair is one float2 so every tangent update is ONE
// v_pk_fma_f32 / v_pk_mul_f32 (two lanes of fp32 work per instruction)
typedef float float2v __attribute__((ext_vector_type(2)));
struct DualF2 {
    float v;
    union {
        float2v t;
        struct { float a, b; };
    };
    DualF2() = default;
    __host__ __device__ constexpr DualF2(double x) : v((float)x), t{0.0f, 0.0f} {}
    __host__ __device__ constexpr DualF2(float x, float ta, float tb) : v(x), t{ta, tb} {}
    __host__ __device__ constexpr DualF2(float x, float2v tt) : v(x), t(tt) {}
};
__device__ __forceinline__ float2v splat2(float f) { return float2v{f, f}; }
__device__ __forceinline__ float2v fma2(float2v a, float2v b, float2v c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ DualF2 mkf2(float v, float2v t) { return DualF2(v, t); }
__device__ __forceinline__ DualF2 mkf2(float v, float a, float b) { return DualF2(v, a, b); }
__device__ __forceinline__ DualF2 operator+(DualF2 x, DualF2 y) { return mkf2(x.v + y.v, x.t + y.t); }
__device__ __forceinline__ DualF2 operator-(DualF2 x, DualF2 y) { return mkf2(x.v - y.v, x.t - y.t); }
__device__ __forceinline__ DualF2 operator-(DualF2 x) { return mkf2(-x.v, -x.t); }
__device__ __forceinline__ DualF2 operator*(DualF2 x, DualF2 y) {
    return mkf2(x.v * y.v, fma2(x.t, splat2(y.v), x.v * y.t));
}
__device__ __forceinline__ DualF2 operator+(DualF2 x, double c) { return mkf2(x.v + (float)c, x.t); }
__device__ __forceinline__ DualF2 operator+(double c, DualF2 x) { return mkf2(x.v + (float)c, x.t); }
__device__ __forceinline__ DualF2 operator-(DualF2 x, double c) { return mkf2(x.v - (float)c, x.t); }
__device__ __forceinline__ DualF2 operator-(double c, DualF2 x) { return mkf2((float)c - x.v, -x.t); }
__device__ __forceinline__ DualF2 operator*(DualF2 x, double c) { const float f = (float)c; return mkf2(x.v * f, x.t * f); }
__device__ __forceinline__ DualF2 operator*(double c, DualF2 x) { const float f = (float)c; return mkf2(x.v * f, x.t * f); }
__device__ __forceinline__ DualF2 operator/(DualF2 x, DualF2 y) {
    const float iy = 1.0f / y.v, q = x.v * iy;
    return mkf2(q, fma2(splat2(-q), y.t, x.t) * iy);
}
__device__ __forceinline__ DualF2 operator/(DualF2 x, double c) { const float ic = (float)(1.0 / c); return mkf2(x.v * ic, x.t * ic); }
__device__ __forceinline__ DualF2 rcp(DualF2 x) { const float r = 1.0f / x.v, nr2 = -r * r; return mkf2(r, x.t * nr2); }
__device__ __forceinline__ float val(DualF2 x) { return x.v; }
__device__ __forceinline__ DualF2 dsqrt(DualF2 x) { const float s = sqrtf(x.v), h = 0.5f / s; return mkf2(s, x.t * h); }
__device__ __forceinline__ DualF2 dexp(DualF2 x) { const float e = expf(x.v); return mkf2(e, x.t * e); }
__device__ __forceinline__ DualF2 dasin(DualF2 x, DualF2 cosv) { const float ic = 1.0f / cosv.v; return mkf2(asinf(x.v), x.t * ic); }
__device__ __forceinline__ DualF2 datan2(DualF2 y, DualF2 x, DualF2 r2) {
    const float ir = 1.0f / r2.v;
    return mkf2(atan2f(y.v, x.v), fma2(splat2(x.v), y.t, splat2(-y.v) * x.t) * ir);
}
// RK4 accumulation step acc + w k (rk4 kernels), packed for DualF2
template <class DT, class ST>
__device__ __forceinline__ DT rk_axpy(ST w, const DT& k, const DT& x) {
    return DT(fma(w, k.v, x.v), fma(w, k.a, x.a), fma(w, k.b, x.b));
}
template <>
__device__ __forceinline__ DualF2 rk_axpy<DualF2, float>(float w, const DualF2& k, const DualF2& x) {
    return mkf2(fmaf(w, k.v, x.v), fma2(splat2(w), k.t, x.t));
}

template <class T> struct V3 { T x, y, z; };

template <class T>
__host__ __device__ __forceinline__ T dot3(const V3<T>& a, const V3<T>& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
template <class T>
__host__ __device__ __forceinline__ V3<T> cross3(const V3<T>& a, const V3<T>& b) {
    return V3<T>{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

// q^-1 (x) [0,v] (x) q  with q = (w,u) (conjugate, not normalised):
//   (w^2 - u.u) v + 2 (u.v) u - 2 w (u x v)
template <class T>
__host__ __device__ __forceinline__ V3<T> rot_body(T w, const V3<T>& u, T ww_uu, const V3<T>& v) {
    T uv2 = 2.0 * dot3(u, v);
    V3<T> c = cross3(u, v);
    T w2 = 2.0 * w;
    return V3<T>{ww_uu * v.x + uv2 * u.x - w2 * c.x,
                 ww_uu * v.y + uv2 * u.y - w2 * c.y,
                 ww_uu * v.z + uv2 * u.z - w2 * c.z};
}
// q (x) [0,v] (x) q^-1 : (w^2 - u.u) v + 2 (u.v) u + 2 w (u x v)
template <class T>
__host__ __device__ __forceinline__ V3<T> rot_world(T w, const V3<T>& u, T ww_uu, const V3<T>& v) {
    T uv2 = 2.0 * dot3(u, v);
    V3<T> c = cross3(u, v);
    T w2 = 2.0 * w;
    return V3<T>{ww_uu * v.x + uv2 * u.x + w2 * c.x,
                 ww_uu * v.y + uv2 * u.y + w2 * c.y,
                 ww_uu * v.z + uv2 * u.z + w2 * c.z};
}

// ---------------------------------------------------------------------------
// kite ODE  x = [v(3) w(3) r(3) q(4)], u = [T dE dR]  -> f[13]
//
// WIND (build extension for wind-field batch sweeps; the reference model has
// no wind, kite.cpp:196 "@todo: add wind"): a constant world-frame wind W
// (wnd[0..2], m/s) makes the aerodynamics -- airspeed, angles, dynamic
// pressure, the rate-damping terms -- see the air-relative body velocity
// v_a = v - q^-1 (x) [0,W] (x) q, while gravity, the tether and the kinematics
// keep the inertial v.  WIND = false is the reference model, instruction for
// instruction.
// ---------------------------------------------------------------------------
template <class T, bool WIND = false>
__host__ __device__ __forceinline__ void kite_rhs(const ModelConst& P, const T* x, const T* u, T* f,
                                                  const double* wnd = nullptr) {
    const V3<T> v{x[0], x[1], x[2]};
    const V3<T> w{x[3], x[4], x[5]};
    const V3<T> r{x[6], x[7], x[8]};
    const T qw = x[9];
    const V3<T> qu{x[10], x[11], x[12]};
    const T thr = u[0], dE = u[1], dR = u[2];
    V3<T> va = v;
    if constexpr (WIND) {
        // the wind is a constant: its rotation multiplies by plain doubles
        // (a dual-typed constant would carry zero tangents through every product)
        const T wwuu = qw * qw - dot3(qu, qu);
        const double W0 = wnd[0], W1 = wnd[1], W2 = wnd[2];
        const T uv2 = 2.0 * (qu.x * W0 + qu.y * W1 + qu.z * W2);
        const T cx = qu.y * W2 - qu.z * W1, cy = qu.z * W0 - qu.x * W2, cz = qu.x * W1 - qu.y * W0;
        const T w2 = 2.0 * qw;
        va = V3<T>{v.x - (wwuu * W0 + uv2 * qu.x - w2 * cx), v.y - (wwuu * W1 + uv2 * qu.y - w2 * cy),
                   v.z - (wwuu * W2 + uv2 * qu.z - w2 * cz)};
    }

    // airspeed, angles (kite.cpp:197-202)
    const T V2 = dot3(va, va);
    const T V = dsqrt(V2);
    const T sb = va.y * rcp(V + 1e-4);             // sin(ss)
    const T cb = dsqrt(1.0 - sb * sb);             // cos(ss) >= 0
    const T ss = dasin(sb, cb);
    const T ax = va.x + 1e-4;
    const T r2a = ax * ax + va.z * va.z;
    const T aoa = datan2(va.z, ax, r2a);
    const T ira = rcp(dsqrt(r2a));
    const T ca = ax * ira, sa = va.z * ira;         // cos/sin(aoa)
    const T qbar = P.half_rho * V2;
    const T qS = qbar * P.S;

    // forces in the wind frame (kite.cpp:204-213)
    const T CLt = P.CL0 + P.CLa * aoa;
    const T CD = P.CD0 + CLt * CLt * P.inv_pieAR;
    const T LIFT = CLt * qS + P.kLq * V * w.y;
    const T DRAG = CD * qS;
    const T SF = (P.CYb * ss + P.CYdr * dR) * qS + (P.CYr * w.z + P.CYp * w.x) * P.kSF * V;

    // Faero = qw_b^-1 [0,-D,0,-L] qw_b with qw_b = q(aoa) q(-ss): rotate by aoa
    // about y, then by -ss about z (kite.cpp:217-226)
    const T a1x = ca * (-DRAG) + sa * LIFT;
    const T a1z = sa * (-DRAG) - ca * LIFT;
    // elevator force q(aoa)^-1 [0,0,0,Zde] q(aoa) (kite.cpp:228-232)
    const T Zde = (-P.CLde) * dE * qS;
    V3<T> Fa{cb * a1x - sa * Zde, sb * a1x + SF, a1z + ca * Zde};

    // quaternion invariants of the state attitude
    const T uu = dot3(qu, qu);
    const T ww_uu = qw * qw - uu;

    // gravity q^-1 [0,0,0,g] q (kite.cpp:237-240): rot_body with v = (0, 0, g)
    // written with its nonzero terms only (x * 0 is not folded for doubles: a
    // dual-typed (0, 0, g) would spend a third of the rotation on zeros)
    const T guv2 = 2.0 * (qu.z * kGravity);
    const T gcx = qu.y * kGravity, gcy = -(qu.x * kGravity);
    const T gw2 = 2.0 * qw;
    const V3<T> Gb{guv2 * qu.x - gw2 * gcx, guv2 * qu.y - gw2 * gcy, ww_uu * kGravity + guv2 * qu.z};

    // tether (kite.cpp:247-265)
    const T d2 = dot3(r, r);
    const T d = dsqrt(d2);
    const T id = rcp(d);
    const V3<T> vi = rot_world(qw, qu, ww_uu, v);           // also r_dot
    const T stretch = d - P.Lt;
    const T hv = rcp(1.0 + dexp(-4.0 * stretch));           // heaviside(d - Lt, 1)
    // R = (Ks Rs + Kd Rd) hv,  Rs = -(d-Lt) r/d,  Rd = -(r/d)(r.vi)/d
    const T coef = -(P.Ks * stretch + P.Kd * dot3(r, vi) * id) * id * hv;
    const V3<T> Rw{coef * r.x, coef * r.y, coef * r.z};
    const V3<T> Rb = rot_body(qw, qu, ww_uu, Rw);

    // v_dot (kite.cpp:268)
    const V3<T> wxv = cross3(w, v);
    f[0] = (Fa.x + thr + Rb.x) * P.inv_mass + Gb.x - wxv.x;
    f[1] = (Fa.y + Rb.y) * P.inv_mass + Gb.y - wxv.y;
    f[2] = (Fa.z + Rb.z) * P.inv_mass + Gb.z - wxv.z;

    // aerodynamic moments (kite.cpp:274-283) in the stability frame
    const T Lr = (P.Cl0 + P.Clb * ss + P.Cldr * dR) * qS * P.b + (P.Clr * w.z + P.Clp * w.x) * P.kRoll * V;
    const T Mp = (P.Cm0 + P.Cma * aoa + P.Cmde * dE) * qS * P.c + P.Cmq * P.kPitch * w.y * V;
    const T Ny = (P.Cn0 + P.Cnb * ss + P.Cndr * dR) * qS * P.b + (P.Cnp * w.x + P.Cnr * w.z) * P.kYaw * V;
    // q(aoa)^-1 [0,L,M,N] q(aoa)  (kite.cpp:293-296)
    const T Max = ca * Lr - sa * Ny;
    const T Maz = sa * Lr + ca * Ny;
    // tether moment r_arm x R_b (kite.cpp:299-300)
    const T Mtx = P.ry * Rb.z - P.rz * Rb.y;
    const T Mty = P.rz * Rb.x - P.rx * Rb.z;
    const T Mtz = P.rx * Rb.y - P.ry * Rb.x;
    // w_dot = J^-1 (Ma + Mt - w x Jw)  (kite.cpp:286-302)
    const V3<T> Jw{P.Ixx * w.x + P.Ixz * w.z, P.Iyy * w.y, P.Ixz * w.x + P.Izz * w.z};
    const V3<T> wxJw = cross3(w, Jw);
    const T m0 = Max + Mtx - wxJw.x;
    const T m1 = Mp + Mty - wxJw.y;
    const T m2 = Maz + Mtz - wxJw.z;
    f[3] = P.Ji00 * m0 + P.Ji02 * m2;
    f[4] = P.Ji11 * m1;
    f[5] = P.Ji02 * m0 + P.Ji22 * m2;

    // r_dot = q [0,v] q^-1 (kite.cpp:308-310)
    f[6] = vi.x; f[7] = vi.y; f[8] = vi.z;

    // q_dot = 0.5 q (x) [0,w] + 0.5 lambda q (q.q - 1), lambda = -5 (kite.cpp:316-317)
    const T nrm = (qw * qw + uu) - 1.0;
    const T lam = -2.5 * nrm;                               // 0.5 * lambda * (|q|^2 - 1)
    const V3<T> uxw = cross3(qu, w);
    f[9]  = -0.5 * dot3(qu, w) + lam * qw;
    f[10] = 0.5 * (qw * w.x + uxw.x) + lam * qu.x;
    f[11] = 0.5 * (qw * w.y + uxw.y) + lam * qu.y;
    f[12] = 0.5 * (qw * w.z + uxw.z) + lam * qu.z;
}

}  // namespace kite
