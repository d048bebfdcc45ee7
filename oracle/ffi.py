"""ctypes front-end of the CPU oracle (oracle/kite_oracle.cpp).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg.  The product (openkite_amd) never imports it.

Also holds the oracle's own view of the kite parameter file and of the
controller configuration the reference ROS node sets up
(src/kite_control/nmpf_node.cpp:30-69, kiteNMPF.cpp:32-34).
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Dict

import numpy as np
import yaml

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "liboracle.so")
REPO = os.path.dirname(_HERE)
DEFAULT_YAML = os.path.join(REPO, "data", "umx_radian.yaml")

# parameter order == kite_oracle.cpp enum KP == include/kite_nmpc/kite_nmpc.h kite_params
PARAM_KEYS = [
    ("geometry", "b"), ("geometry", "c"), ("geometry", "AR"), ("geometry", "S"),
    ("geometry", "lam"), ("geometry", "St"), ("geometry", "lt"), ("geometry", "Sf"),
    ("geometry", "lf"), ("geometry", "Xac"),
    ("inertia", "mass"), ("inertia", "Ixx"), ("inertia", "Iyy"), ("inertia", "Izz"), ("inertia", "Ixz"),
    ("aerodynamic", "CL0"), ("aerodynamic", "CL0_tail"), ("aerodynamic", "CLa_total"),
    ("aerodynamic", "CLa_wing"), ("aerodynamic", "CLa_tail"), ("aerodynamic", "e_oswald"),
    ("aerodynamic", "CD0_total"), ("aerodynamic", "CD0_wing"), ("aerodynamic", "CD0_tail"),
    ("aerodynamic", "CYb"), ("aerodynamic", "CYb_vtail"), ("aerodynamic", "Cm0"), ("aerodynamic", "Cma"),
    ("aerodynamic", "Cn0"), ("aerodynamic", "Cnb"), ("aerodynamic", "Cl0"), ("aerodynamic", "Clb"),
    ("aerodynamic", "CLq"), ("aerodynamic", "Cmq"), ("aerodynamic", "CYr"), ("aerodynamic", "Cnr"),
    ("aerodynamic", "Clr"), ("aerodynamic", "CYp"), ("aerodynamic", "Clp"), ("aerodynamic", "Cnp"),
    ("aerodynamic", "CLde"), ("aerodynamic", "CYdr"), ("aerodynamic", "Cmde"), ("aerodynamic", "Cndr"),
    ("aerodynamic", "Cldr"), ("aerodynamic", "CDde"),
    ("tether", "length"), ("tether", "Ks"), ("tether", "Kd"), ("tether", "rx"), ("tether", "ry"),
    ("tether", "rz"),
]
assert len(PARAM_KEYS) == 52


def load_params(path: str = DEFAULT_YAML) -> np.ndarray:
    with open(path) as f:
        doc = yaml.safe_load(f)
    return np.array([float(doc[a][b]) for a, b in PARAM_KEYS], dtype=np.float64)


def node_config(N: int = 20, dt: float = 0.05) -> Dict:
    """Controller configuration of the reference ROS node (nmpf_node.cpp:30-69)."""
    inf = math.inf
    sat = math.radians(7.0)
    return dict(
        N=N, dt=dt,
        Q=[1e3, 1e3, 1e4], R=[1e-4, 1e-1, 1e-1, 1e-3], W=1e-3,       # kiteNMPF.cpp:32-34
        Sx=[0.1, 1 / 3.0, 1 / 3.0, 1 / 2.0, 1 / 5.0, 1 / 2.0, 1 / 3.0, 1 / 3.0, 1 / 3.0,
            1.0, 1.0, 1.0, 1.0, 1 / 6.28, 1 / 6.28],
        Su=[1 / 0.15, 1 / 0.2618, 1 / 0.2618, 1 / 5.0],
        lbx=[2.0, -inf, -inf, -4 * math.pi, -4 * math.pi, -4 * math.pi, -inf, -inf, -inf,
             -1.01, -1.01, -1.01, -1.01, -inf, -inf],
        ubx=[inf, inf, inf, 4 * math.pi, 4 * math.pi, 4 * math.pi, inf, inf, inf,
             1.01, 1.01, 1.01, 1.01, inf, inf],
        lbu=[0.1, -sat, -sat, -5.0], ubu=[0.15, sat, sat, 5.0],
        vref=4.0,
        path_R=2.65, path_alt=0.0,
        path_q=[math.cos(math.pi / 8), 0.0, math.sin(math.pi / 8), 0.0],
        flex=0.78, min_speed=2.1,
        delay=0.0, delay_steps=16,    # node transport delay 0.1 s (nmpf_node.cpp:74); 0 = KiteNMPF alone
        qp_form=0 if N == 20 else 1,  # the product's qp_kernel 0 (auto): N == 20 condensed QP + lazy
                                      # state rows (qp_form 0, qp_kernel 2), otherwise the
                                      # multiple-shooting QP (qp_form 1, qp_kernel 3)
        soft_weight=1e3, lm=10.0,     # kite_nmpc_default_config qp_soft_weight, qp_lm
        qp_rec=1e-6 if N == 20 else 0.0,   # condensed IPM: recursive residuals above 1e-6 as k_qp_tiled
                                           # (qp_kernel 2 at N = 20); 0 = exact each iteration (k_qp,
                                           # k_qp_lds: qp_kernel 1, other horizons)
    )


def cfg_vector(c: Dict) -> np.ndarray:
    v = [c["dt"], *c["Q"], *c["R"], c["W"], *c["Sx"], *c["Su"], *c["lbx"], *c["ubx"],
         *c["lbu"], *c["ubu"], c["vref"], c["path_R"], c["path_alt"], *c["path_q"],
         c["flex"], c["min_speed"], c.get("delay", 0.0), c.get("delay_steps", 16), c.get("qp_form", 1),
         c.get("soft_weight", 1e3), c.get("lm", 10.0), c.get("path_K", 0)]
    F = np.zeros((3, 17))
    if c.get("path_K", 0):
        F[:] = np.asarray(c["path_fourier"], dtype=np.float64).reshape(3, 17)
    a = np.concatenate([np.array(v, dtype=np.float64), F.reshape(-1),
                        np.array([c.get("qp_rec", 1e-6 if c.get("N", 20) == 20 else 0.0)], dtype=np.float64)])
    assert a.size == 133
    return a


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"oracle not built: {LIB_PATH} (run make -C oracle)")
        L = ctypes.CDLL(LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int32)
        i = ctypes.c_int
        d = ctypes.c_double
        sig = {
            "orc_rhs": (None, [dp, dp, dp, dp]),
            "orc_rhs_aug": (None, [dp, dp, dp, dp]),
            "orc_rhs_jac_cs": (None, [dp, dp, dp, dp]),
            "orc_rhs_jac_ad": (None, [dp, dp, dp, dp]),
            "orc_ekf_step": (None, [dp, dp, dp, d, dp, dp, dp, dp]),
            "orc_colloc_eval": (None, [dp, dp, i, dp, dp, dp, dp]),
            "orc_rk4": (None, [dp, dp, dp, d, i, dp]),
            "orc_rk4_sens": (None, [dp, dp, dp, d, i, dp, dp, dp]),
            "orc_rk4_sens_cs": (None, [dp, dp, dp, d, i, dp, dp]),
            "orc_path": (None, [dp, d, dp, dp]),
            "orc_closest_point": (d, [dp, dp, d]),
            "orc_build_qp": (i, [dp, dp, i, i, dp, dp, dp, dp, dp, dp, dp, dp, dp, dp, dp]),
            "orc_qp_solve": (d, [i, i, dp, dp, dp, dp, dp, dp, i, dp]),
            "orc_prologue": (i, [dp, dp, i, i, dp, i, i, dp, dp, dp]),
            "orc_msqp_solve": (d, [dp, dp, i, i, dp, dp, i, dp, ip]),
            "orc_msqp_solve_pert": (d, [dp, dp, i, i, dp, dp, i, d, i, dp, ip]),
            "orc_set_wind": (None, [dp]),
            "orc_set_wind_batch": (None, [dp, i]),
            "orc_set_ms_z0": (None, [d]),
            "orc_set_ipm_z0": (None, [d]),
            "orc_set_ipm_gondzio": (None, [i]),
            "orc_set_ipm_study": (None, [d, d]),
            "orc_gondzio_solves": (ctypes.c_longlong, []),
            "orc_get_ipm_z0": (d, []),
            "orc_get_ms_z0": (d, []),
            "orc_msqp_build": (i, [dp, dp, i, i, dp, dp, dp, dp, dp, dp, dp, dp, dp, dp, dp]),
            "orc_rti_step": (None, [dp, dp, i, i, i, i, i, i, dp, dp, dp, dp, dp, ip, i, ip]),
            "orc_set_sqp": (None, [d, i]),
            "orc_sqp_step": (None, [dp, dp, i, i, i, i, i, i, i, d, dp, dp, dp, dp, dp, ip, i, ip, dp]),
            "orc_traj_cost": (d, [dp, i, dp, dp]),
            "orc_cheb_points": (None, [i, dp]),
            "orc_cheb_D": (None, [i, dp]),
            "orc_cheb_weights": (None, [i, dp]),
            "orc_cheb_compD": (None, [i, i, dp]),
            "orc_cheb_expansion": (d, [dp, i, d]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _p(a):
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def rhs(kp, x13, u3):
    f = np.zeros(13)
    lib().orc_rhs(_p(kp), _p(_f64(x13)), _p(_f64(u3)), _p(f))
    return f


def rhs_aug(kp, x15, u4):
    f = np.zeros(15)
    lib().orc_rhs_aug(_p(kp), _p(_f64(x15)), _p(_f64(u4)), _p(f))
    return f


COLLOC_KEYS = ["poly_order", "num_segments", "use_R", "t0", "tf", "Q", "R", "W", "vref", "mayer_scale", "Sx", "Su",
               "path_radius", "path_altitude", "path_q"]


def colloc_vector(c: Dict) -> np.ndarray:
    v = []
    for k in COLLOC_KEYS:
        x = c[k]
        v.extend(x if isinstance(x, (list, tuple, np.ndarray)) else [x])
    F = np.zeros((3, 17))
    K = int(c.get("path_harmonics", 0))
    if K:
        F[:] = np.asarray(c["path_fourier"], dtype=np.float64).reshape(3, 17)
    a = np.concatenate([np.array(v, dtype=np.float64), [float(K)], F.reshape(-1)])
    assert a.size == 92
    return a


def colloc_eval(kp, c: Dict, z, jac=False):
    """Reference collocation G, J (and Jacobian blocks) at points z (count x nz)."""
    z = _f64(z).reshape(-1, (c["poly_order"] * c["num_segments"] + 1) * 19)
    cnt, n = z.shape[0], c["poly_order"] * c["num_segments"] + 1
    G = np.zeros((cnt, n * 15)); J = np.zeros(cnt)
    Jb = np.zeros((cnt, n, 15, 19)) if jac else None
    lib().orc_colloc_eval(_p(kp), _p(colloc_vector(c)), cnt, _p(z), _p(G), _p(J), None if Jb is None else _p(Jb))
    return (G, J, Jb) if jac else (G, J)


def ekf_step(kp, x13, u3, dt, P, z7, W, V):
    """KiteEKF propagate (+ update when z7 is not None) for one kite; returns (x, P)."""
    x = _f64(x13).copy(); Pm = _f64(P).reshape(13, 13).copy()
    lib().orc_ekf_step(_p(kp), _p(x), _p(_f64(u3)), float(dt), _p(Pm), None if z7 is None else _p(_f64(z7)),
                       _p(_f64(W)), _p(_f64(V)))
    return x, Pm


def rhs_jac(kp, x13, u3, method="ad"):
    J = np.zeros((13, 16))
    fn = lib().orc_rhs_jac_ad if method == "ad" else lib().orc_rhs_jac_cs
    fn(_p(kp), _p(_f64(x13)), _p(_f64(u3)), _p(J))
    return J


def rk4(kp, x15, u4, h, M=1):
    xo = np.zeros(15)
    lib().orc_rk4(_p(kp), _p(_f64(x15)), _p(_f64(u4)), float(h), int(M), _p(xo))
    return xo


def rk4_sens(kp, x15, u4, h, M=1):
    xo = np.zeros(15); A = np.zeros((15, 15)); B = np.zeros((15, 4))
    lib().orc_rk4_sens(_p(kp), _p(_f64(x15)), _p(_f64(u4)), float(h), int(M), _p(xo), _p(A), _p(B))
    return xo, A, B


def rk4_sens_cs(kp, x15, u4, h, M=1):
    A = np.zeros((15, 15)); B = np.zeros((15, 4))
    lib().orc_rk4_sens_cs(_p(kp), _p(_f64(x15)), _p(_f64(u4)), float(h), int(M), _p(A), _p(B))
    return A, B


def path(cfgv, theta):
    P = np.zeros(3); dP = np.zeros(3)
    lib().orc_path(_p(cfgv), float(theta), _p(P), _p(dP))
    return P, dP


def closest_point(cfgv, pos, guess=0.0):
    return lib().orc_closest_point(_p(cfgv), _p(_f64(pos)), float(guess))


def build_qp(kp, cfgv, N, M, X, U, want_G=False):
    """Condensed QP of the oracle (scaled variables, oracle column order);
    want_G: also G = d x / d dw, shape (N + 1, 15, n) (unscaled dw = D w)."""
    n = 4 * N + 2
    mmax = 2 * N
    H = np.zeros((n, n)); h = np.zeros(n); lb = np.zeros(n); ub = np.zeros(n)
    C = np.zeros((mmax, n)); c = np.zeros(mmax); D = np.zeros(n); g = np.zeros((N + 1, 15))
    G = np.zeros((N + 1, 15, n)) if want_G else None
    m = lib().orc_build_qp(_p(kp), _p(cfgv), N, M, _p(_f64(X)), _p(_f64(U)), _p(H), _p(h), _p(lb),
                           _p(ub), _p(C), _p(c), _p(D), _p(g), _p(G) if want_G else None)
    return dict(H=H, h=h, lb=lb, ub=ub, C=C[:m].copy(), c=c[:m].copy(), D=D, g=g, m=m, G=G)


def qp_solve(H, h, lb, ub, C, c, K):
    n = H.shape[0]
    m = C.shape[0]
    w = np.zeros(n)
    kkt = lib().orc_qp_solve(n, m, _p(_f64(H)), _p(_f64(h)), _p(_f64(lb)), _p(_f64(ub)),
                             _p(_f64(C.reshape(-1)) if m else np.zeros(1)),
                             _p(_f64(c) if m else np.zeros(1)), int(K), _p(w))
    return w, kkt


def ms_trace():
    """Per-iteration (r, mu, affine step, sigma, step) of the last msqp_solve on
    this thread (debug aid)."""
    L = lib()
    buf = np.zeros(64 * 5)
    L.orc_ms_trace.restype = ctypes.c_int
    n = L.orc_ms_trace(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    return buf[:5 * n].reshape(n, 5)


def msqp_solve(kp, cfgv, N, M, X, U, K):
    """Multiple-shooting QP (qp_form 1) at the linearisation point (X, U) after
    the prologue; returns (v, kkt, iterations), v = [dx_0 du_0 ... dx_N] scaled."""
    nv = (N + 1) * 15 + N * 4
    v = np.zeros(nv)
    it = np.zeros(1, dtype=np.int32)
    kkt = lib().orc_msqp_solve(_p(kp), _p(cfgv), N, M, _p(_f64(X)), _p(_f64(U)), int(K), _p(v),
                               it.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    return v, kkt, int(it[0])


def msqp_solve_perturbed(kp, cfgv, N, M, X, U, K, eps, seed):
    """msqp_solve with the QP data (A, B, d, J, r, Rh, rho) perturbed by a
    relative eps * N(0, 1) per element (fixed seed): the QP's sensitivity
    envelope under rounding-level differences."""
    nv = (N + 1) * 15 + N * 4
    v = np.zeros(nv)
    it = np.zeros(1, dtype=np.int32)
    kkt = lib().orc_msqp_solve_pert(_p(kp), _p(cfgv), N, M, _p(_f64(X)), _p(_f64(U)), int(K), float(eps),
                                    int(seed), _p(v), it.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    return v, kkt, int(it[0])


def set_ms_z0(z0: float) -> float:
    """Start multiplier of the oracle's multiple-shooting IPM (tools only; the
    GPU kernel has its own constant RIC_Z0).  Returns the previous value."""
    L = lib()
    old = L.orc_get_ms_z0()
    L.orc_set_ms_z0(float(z0))
    return old


def set_ipm_gondzio(k: int) -> None:
    """Study switch: up to k Gondzio centrality correctors in the oracle's
    condensed IPM (tools only; 0 = the product rule, which the GPU kernels
    implement)."""
    lib().orc_set_ipm_gondzio(int(k))


def set_ipm_study(tau: float = 0.995, s0: float = 0.1) -> None:
    """Study switches: the condensed IPM's step-to-boundary floor and start
    slack (tools only; the defaults are the product constants)."""
    lib().orc_set_ipm_study(float(tau), float(s0))


def gondzio_solves() -> int:
    """Corrector solves since the last set_ipm_gondzio (tools only)."""
    return int(lib().orc_gondzio_solves())


def set_ipm_z0(z0: float) -> float:
    """Start multiplier of the oracle's condensed IPM (tools only; the GPU
    kernels have their own constant IPM_Z0).  Returns the previous value."""
    L = lib()
    old = L.orc_get_ipm_z0()
    L.orc_set_ipm_z0(float(z0))
    return old


def msqp_build(kp, cfgv, N, M, X, U):
    """The multiple-shooting QP's data (scaled): dict of A, B, d, J, r, Rh, rho, lo, hi."""
    nv = (N + 1) * 15 + N * 4
    o = dict(A=np.zeros((N, 15, 15)), B=np.zeros((N, 15, 4)), d=np.zeros((N, 15)), J=np.zeros((N + 1, 4, 15)),
             r=np.zeros((N + 1, 4)), Rh=np.zeros(4), rho=np.zeros((N, 4)), lo=np.zeros(nv), hi=np.zeros(nv))
    lib().orc_msqp_build(_p(kp), _p(cfgv), N, M, _p(_f64(X)), _p(_f64(U)), *(_p(o[k]) for k in
                         ("A", "B", "d", "J", "r", "Rh", "rho", "lo", "hi")))
    return o


def prologue(kp, cfgv, N, M, x0, X, U, warm, shift=1):
    X = _f64(X).copy(); U = _f64(U).copy(); x0o = np.zeros(15)
    st = lib().orc_prologue(_p(kp), _p(cfgv), N, M, _p(_f64(x0)), int(warm), int(shift), _p(X), _p(U), _p(x0o))
    return st, X, U, x0o


def rti_step(kp, cfgv, N, M, K, x0, X, U, warm, shift=1, nthreads=0, iters=None, wind=None):
    """Batched RTI step.  x0 (B,15); X (B,N+1,15) and U (B,N,4) updated in place.
    iters (optional int32 array of B): QP interior-point iterations per kite (the
    condensed form counts the last re-solve only).  wind (optional (B,3)): per-kite
    world-frame wind (build extension; None = the reference model)."""
    B = x0.shape[0]
    assert X.shape == (B, N + 1, 15) and U.shape == (B, N, 4)
    assert X.dtype == np.float64 and U.dtype == np.float64 and X.flags["C_CONTIGUOUS"] and U.flags["C_CONTIGUOUS"]
    u0 = np.zeros((B, 4)); diag = np.zeros((B, 6)); status = np.zeros(B, dtype=np.int32)
    ip = ctypes.POINTER(ctypes.c_int32)
    wv = None if wind is None else _f64(np.asarray(wind, dtype=np.float64).reshape(B, 3))
    lib().orc_set_wind_batch(None if wv is None else _p(wv), B)
    try:
        lib().orc_rti_step(_p(kp), _p(cfgv), N, M, K, B, int(warm), int(shift), _p(_f64(x0)), _p(X), _p(U),
                           _p(u0), _p(diag), status.ctypes.data_as(ip), int(nthreads),
                           None if iters is None else iters.ctypes.data_as(ip))
    finally:
        lib().orc_set_wind_batch(None, 0)
    return u0, diag, status


def sqp_step(kp, cfgv, N, M, K, x0, X, U, warm, maxit, tol, shift=1, nthreads=0, wind=None):
    """Gauss-Newton SQP to convergence at one sampling instant (orc_sqp_step):
    the RTI step, then re-linearisations at the same processed measurement with
    the theta box fixed at it, until the full step (scaled inf-norm) is below
    tol or maxit iterations.  Returns u0, diag, status, sqp iterations, last step."""
    B = x0.shape[0]
    assert X.shape == (B, N + 1, 15) and U.shape == (B, N, 4)
    assert X.dtype == np.float64 and U.dtype == np.float64 and X.flags["C_CONTIGUOUS"] and U.flags["C_CONTIGUOUS"]
    u0 = np.zeros((B, 4)); diag = np.zeros((B, 6)); status = np.zeros(B, dtype=np.int32)
    its = np.zeros(B, dtype=np.int32); step = np.zeros(B)
    ip = ctypes.POINTER(ctypes.c_int32)
    wv = None if wind is None else _f64(np.asarray(wind, dtype=np.float64).reshape(B, 3))
    lib().orc_set_wind_batch(None if wv is None else _p(wv), B)
    try:
        lib().orc_sqp_step(_p(kp), _p(cfgv), N, M, K, B, int(warm), int(shift), int(maxit), float(tol),
                           _p(_f64(x0)), _p(X), _p(U), _p(u0), _p(diag), status.ctypes.data_as(ip),
                           int(nthreads), its.ctypes.data_as(ip), _p(step))
    finally:
        lib().orc_set_wind_batch(None, 0)
    return u0, diag, status, its, step


def set_wind(w3):
    """World-frame wind of this thread's single-kite oracle calls (rhs, rk4,
    rk4_sens, prologue, ...); None = no wind (the reference model)."""
    lib().orc_set_wind(None if w3 is None else _p(_f64(np.asarray(w3, dtype=np.float64).reshape(3))))


def traj_cost(cfgv, N, X, U):
    return lib().orc_traj_cost(_p(cfgv), N, _p(_f64(X)), _p(_f64(U)))


def cheb_points(n):
    x = np.zeros(n + 1); lib().orc_cheb_points(n, _p(x)); return x


def cheb_D(n):
    D = np.zeros((n + 1, n + 1)); lib().orc_cheb_D(n, _p(D)); return D


def cheb_weights(n):
    w = np.zeros(n + 1); lib().orc_cheb_weights(n, _p(w)); return w


def cheb_compD(P, S):
    m = S * P + 1
    D = np.zeros((m, m)); lib().orc_cheb_compD(P, S, _p(D)); return D


def cheb_expansion(coef, x):
    c = _f64(coef)
    return lib().orc_cheb_expansion(_p(c), c.size, float(x))


# ---- synthetic benchmark inputs --------------------------
BASE_STATE = np.array([4.4, 0.44, 1.73, 0.81, -1.73, -1.53, -0.46, -2.68, 0.64,
                       -0.0289, 0.1587, 0.4304, 0.8881])   # launch/simulator.launch:3
SEED0 = 20261015


def synthetic_states(B: int, seed0: int = SEED0, offset: int = 0) -> np.ndarray:
    """Per-instance seeded perturbations of the in-flight state (13 kite states)."""
    out = np.zeros((B, 13))
    for b in range(B):
        rng = np.random.default_rng(seed0 + offset + b)
        x = BASE_STATE.copy()
        x[0:3] += rng.uniform(-0.5, 0.5, 3)
        x[3:6] += rng.uniform(-0.3, 0.3, 3)
        x[6:9] += rng.uniform(-0.05, 0.05, 3)
        axis = rng.normal(size=3)
        axis /= np.linalg.norm(axis)
        ang = math.radians(5.0) * rng.uniform(0, 1)
        dq = np.array([math.cos(ang / 2), *(math.sin(ang / 2) * axis)])
        q = x[9:13]
        # Hamilton product q (x) dq, then normalise
        w1, v1 = q[0], q[1:]
        w2, v2 = dq[0], dq[1:]
        qn = np.array([w1 * w2 - v1 @ v2, *(np.cross(v1, v2) + w1 * v2 + w2 * v1)])
        x[9:13] = qn / np.linalg.norm(qn)
        out[b] = x
    return out
