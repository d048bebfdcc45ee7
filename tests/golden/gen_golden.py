#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ (run here, never on the GPU box).

An independent symbolic restatement of the openKITE kite model, written with
sympy in the reference's own form (literal w-first quaternion products
kitemath.cpp:9-29, the ODE of kite.cpp:197-317, the augmentation of
kiteNMPF.cpp:62-79, the rotated path of nmpf_node.cpp:30-40), evaluated with
mpmath at 50 significant digits.  It pins:

  * f(x,u) and the exact Jacobian d f / d [x,u]  (sympy.diff)
  * one RK4 interval with M substeps (kitemath.cpp:36-51) and its exact
    sensitivities (the RK4 map differentiated symbolically stage by stage)
  * Chebyshev-Gauss-Lobatto D, Clenshaw-Curtis weights, composite D and the
    Chebyshev expansion (chebyshev.hpp:113-232, kitemath.h:50-72)
  * the path P(theta) and dP/dtheta
  * the collocation residual G and cost J of the reference's full_generics
    test NLP at its own 209-vector (chebyshev.hpp:241-333)
  * the RTI objective (the reference's Lagrange / Mayer terms with the node's
    weights and scaling) on the shooting grid at seeded plans

Inputs are the known-answer states of the reference tests plus
seeded perturbations of the in-flight state of launch/simulator.launch:3.
The reference itself cannot run here (CasADi / IPOPT / ROS absent), so these
fixtures + textbook values are the parity pin of the CPU oracle.

Usage:  python tests/golden/gen_golden.py   (writes kite_golden.json)
"""
from __future__ import annotations

import json
import math
import os

import mpmath as mp
import numpy as np
import sympy as sp
import yaml

mp.mp.dps = 50
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def load_yaml(path):
    with open(path) as f:
        return yaml.safe_load(f)


def qmul(a, b):
    s1, v1 = a[0], sp.Matrix(a[1:4])
    s2, v2 = b[0], sp.Matrix(b[1:4])
    s = s1 * s2 - v1.dot(v2)
    v = v1.cross(v2) + s1 * v2 + s2 * v1
    return [s, v[0], v[1], v[2]]


def qinv(a):
    return [a[0], -a[1], -a[2], -a[3]]


def kite_symbolic(prm):
    """Returns (x13, u3, f13) sympy objects following kite.cpp:197-317."""
    g = sp.Rational("9.80665")
    ro = sp.Rational("1.2985")
    P = {k: sp.Rational(repr(float(v))) for sec in ("geometry", "inertia", "aerodynamic", "tether")
         for k, v in prm[sec].items()}
    b, c, AR, S = P["b"], P["c"], P["AR"], P["S"]
    Mass, Ixx, Iyy, Izz, Ixz = P["mass"], P["Ixx"], P["Iyy"], P["Izz"], P["Ixz"]
    x = sp.symbols("x0:13", real=True)
    u = sp.symbols("u0:3", real=True)
    v = sp.Matrix(x[0:3]); w = sp.Matrix(x[3:6]); r = sp.Matrix(x[6:9]); q = list(x[9:13])
    T, dE, dR = u
    V = sp.sqrt(v.dot(v))
    V2 = v.dot(v)
    ss = sp.asin(v[1] / (V + sp.Rational(1, 10000)))
    aoa = sp.atan2(v[2], v[0] + sp.Rational(1, 10000))
    dyn = sp.Rational(1, 2) * ro * V2
    CD = P["CD0_total"] + (P["CL0"] + P["CLa_total"] * aoa) ** 2 / (sp.pi * P["e_oswald"] * AR)
    LIFT = (P["CL0"] + P["CLa_total"] * aoa) * dyn * S + (sp.Rational(1, 4) * P["CLq"] * c * S * ro) * V * w[1]
    DRAG = CD * dyn * S
    SF = (P["CYb"] * ss + P["CYdr"] * dR) * dyn * S + sp.Rational(1, 4) * (P["CYr"] * w[2] + P["CYp"] * w[0]) * (b * ro * S) * V
    q_aoa = [sp.cos(aoa / 2), 0, sp.sin(aoa / 2), 0]
    q_ss = [sp.cos(-ss / 2), 0, 0, sp.sin(-ss / 2)]
    qwb = qmul(q_aoa, q_ss)
    F = qmul(qmul(qinv(qwb), [0, -DRAG, 0, -LIFT]), qwb)
    Fa = sp.Matrix(F[1:4])
    Zde = (-P["CLde"]) * dE * dyn * S
    FE = qmul(qmul(qinv(q_aoa), [0, 0, 0, Zde]), q_aoa)
    Fa = Fa + sp.Matrix(FE[1:4]) + sp.Matrix([0, SF, 0])
    G = qmul(qmul(qinv(q), [0, 0, 0, g]), q)
    Gb = sp.Matrix(G[1:4])
    d_ = sp.sqrt(r.dot(r))
    Rv = d_ - P["length"]
    Rs = -Rv * (r / d_)
    VI = qmul(qmul(q, [0, v[0], v[1], v[2]]), qinv(q))
    vi = sp.Matrix(VI[1:4])
    Rd = (-r / d_) * r.dot(vi) / d_
    hv = 1 / (1 + sp.exp(-4 * (d_ - P["length"])))
    R = (P["Ks"] * Rs + P["Kd"] * Rd) * hv
    RB = qmul(qmul(qinv(q), [0, R[0], R[1], R[2]]), q)
    Rb = sp.Matrix(RB[1:4])
    vdot = (Fa + sp.Matrix([T, 0, 0]) + Rb) / Mass + Gb - w.cross(v)
    L = (P["Cl0"] + P["Clb"] * ss + P["Cldr"] * dR) * dyn * S * b + (P["Clr"] * w[2] + P["Clp"] * w[0]) * (sp.Rational(1, 4) * ro * b ** 2 * S) * V
    M = (P["Cm0"] + P["Cma"] * aoa + P["Cmde"] * dE) * dyn * S * c + P["Cmq"] * (sp.Rational(1, 4) * S * c ** 2 * ro) * w[1] * V
    N = (P["Cn0"] + P["Cnb"] * ss + P["Cndr"] * dR) * dyn * S * b + (P["Cnp"] * w[0] + P["Cnr"] * w[2]) * (sp.Rational(1, 4) * S * b ** 2 * ro) * V
    J = sp.Matrix([[Ixx, 0, Ixz], [0, Iyy, 0], [Ixz, 0, Izz]])
    TR = qmul(qmul(qinv(q_aoa), [0, L, M, N]), q_aoa)
    Ma = sp.Matrix(TR[1:4])
    arm = sp.Matrix([P.get("rx", 0), P.get("ry", 0), P.get("rz", 0)])
    Mt = arm.cross(Rb)
    wdot = J.inv() * (Ma + Mt - w.cross(J * w))
    rdot = vi
    qw = qmul(q, [0, w[0], w[1], w[2]])
    qq = sum(qi * qi for qi in q)
    qdot = [sp.Rational(1, 2) * qw[i] + sp.Rational(1, 2) * (-5) * q[i] * (qq - 1) for i in range(4)]
    f = list(vdot) + list(wdot) + list(rdot) + qdot
    return x, u, f


def to_mp(a):
    return [mp.mpf(repr(float(v))) for v in a]


def mpl(vals):
    return [float(v) for v in vals]


def main():
    prm = load_yaml(os.path.join(REPO, "data", "umx_radian.yaml"))
    x, u, f = kite_symbolic(prm)
    xs = list(x) + list(u)
    fn = sp.lambdify(xs, f, modules="mpmath")
    Jsym = sp.Matrix(f).jacobian(sp.Matrix(xs))
    jfn = sp.lambdify(xs, Jsym, modules="mpmath")

    def f_mp(xv, uv):
        return [mp.mpf(t) for t in fn(*xv, *uv)]

    def jac_mp(xv, uv):
        Jm = jfn(*xv, *uv)
        return [[mp.mpf(Jm[i, j]) for j in range(16)] for i in range(13)]

    # ---- known-answer states ----------------------------------
    states = []
    states.append(("kite_control_test.cpp:252-256", [1.5, 0, 0, 0, 0, 0, 0, 1.0, 0, 1, 0, 0, 0], [0.1, 0, 0]))
    states.append(("kite_model_test.cpp:58-60", [6.1977743, -0.028407148, 0.91815942, 0.29763089, -2.2052198,
                                                 -0.14827499, -0.41624807, -2.2601052, 1.2903439, 0.035646195,
                                                 -0.069986094, 0.82660637, 0.55727089], [0.1, 0, 0]))
    states.append(("kite_control_test.cpp:28-29", [4.318732, 0.182552, 0.254833, 1.85435, -0.142882, -0.168359,
                                                   -0.229383, -0.0500282, -0.746832, 0.189409, -0.836349, -0.48178,
                                                   0.180367], [0.0, 0.0, 0.0]))
    states.append(("kite_control_test.cpp:52-55", [6.0026, -0.3965, 0.1705, 0.4414, -0.2068, 0.9293, 1.4634, -3.1765,
                                                   -1.7037, -0.5486, -0.2354, -0.2922, -0.7471], [0.0, 0.0, 0.0]))
    base = [4.4, 0.44, 1.73, 0.81, -1.73, -1.53, -0.46, -2.68, 0.64, -0.0289, 0.1587, 0.4304, 0.8881]
    states.append(("launch/simulator.launch:3", base, [0.125, 0.0, 0.0]))
    rng = np.random.default_rng(20261015)
    for i in range(32):
        xv = np.array(base, dtype=float)
        xv[0:3] += rng.uniform(-1.0, 1.0, 3)
        xv[3:6] += rng.uniform(-0.6, 0.6, 3)
        xv[6:9] += rng.uniform(-0.3, 0.3, 3)
        xv[9:13] += rng.uniform(-0.05, 0.05, 4)          # |q| != 1 on purpose (exercises the lambda term)
        uv = [rng.uniform(0.1, 0.15), rng.uniform(-0.12, 0.12), rng.uniform(-0.12, 0.12)]
        states.append((f"seeded[{i}] seed=20261015", [float(t) for t in xv], uv))

    rhs_cases = []
    for src, xv, uv in states:
        xm, um = to_mp(xv), to_mp(uv)
        fv = f_mp(xm, um)
        J = jac_mp(xm, um)
        rhs_cases.append(dict(source=src, x=xv, u=uv, f=mpl(fv), J=[mpl(row) for row in J]))

    # ---- RK4 intervals with exact sensitivities -------------------------------
    def aug_f(x15, u4):
        fk = f_mp(x15[:13], u4[:3])
        return fk + [x15[14], u4[3]]

    def aug_J(x15, u4):
        Jk = jac_mp(x15[:13], u4[:3])
        A = [[mp.mpf(0)] * 15 for _ in range(15)]
        Bm = [[mp.mpf(0)] * 4 for _ in range(15)]
        for i in range(13):
            for j in range(13):
                A[i][j] = Jk[i][j]
            for j in range(3):
                Bm[i][j] = Jk[i][13 + j]
        A[13][14] = mp.mpf(1)
        Bm[14][3] = mp.mpf(1)
        return A, Bm

    def matmul(Am, Bm):
        n, m, p = len(Am), len(Bm), len(Bm[0])
        return [[mp.fsum(Am[i][k] * Bm[k][j] for k in range(m)) for j in range(p)] for i in range(n)]

    def rk4_sens(x15, u4, h, M):
        """RK4 and its exact derivative (chain rule through the 4 stages)."""
        xv = list(x15)
        S = [[mp.mpf(1 if i == j else 0) for j in range(19)] for i in range(15)]   # d x / d [x0 u]
        Eu = [[mp.mpf(0)] * 19 for _ in range(4)]
        for j in range(4):
            Eu[j][15 + j] = mp.mpf(1)
        for _ in range(M):
            ks, dks = [], []
            xs, Ss = xv, S
            for st in range(4):
                k = aug_f(xs, u4)
                A, Bm = aug_J(xs, u4)
                dk = [[a + b for a, b in zip(r1, r2)] for r1, r2 in zip(matmul(A, Ss), matmul(Bm, Eu))]
                ks.append(k); dks.append(dk)
                if st < 3:
                    c = h / 2 if st < 2 else h
                    xs = [xi + c * ki for xi, ki in zip(xv, k)]
                    Ss = [[S[i][j] + c * dk[i][j] for j in range(19)] for i in range(15)]
            xv = [xv[i] + (h / 6) * (ks[0][i] + 2 * ks[1][i] + 2 * ks[2][i] + ks[3][i]) for i in range(15)]
            S = [[S[i][j] + (h / 6) * (dks[0][i][j] + 2 * dks[1][i][j] + 2 * dks[2][i][j] + dks[3][i][j])
                  for j in range(19)] for i in range(15)]
        return xv, S

    rk4_cases = []
    h_int, M_int = mp.mpf("0.05"), 2
    for idx in [0, 1, 4] + list(range(5, 13)):
        src, xv, uv = states[idx]
        x15 = to_mp(list(xv) + [0.3, -0.4])
        u4 = to_mp(list(uv) + [0.7])
        xo, S = rk4_sens(x15, u4, h_int / M_int, M_int)
        rk4_cases.append(dict(source=src, x=mpl(x15), u=mpl(u4), tf=float(h_int), M=M_int, xnext=mpl(xo),
                              A=[mpl(r[:15]) for r in S], B=[mpl(r[15:]) for r in S]))
    # the reference's own RK4 call: ODESolver rk4 one step of tf = 7 s (kite_model_test.cpp:58-75)
    src, xv, uv = states[1]
    x15 = to_mp(list(xv) + [0.0, 0.0])
    u4 = to_mp(list(uv) + [0.0])
    xo, _ = rk4_sens(x15, u4, mp.mpf(7), 1)
    rk4_ref_call = dict(source="kite_model_test.cpp:58-75 rk4_solver.solve(init_state, control, 7.0)",
                        x=mpl(x15), u=mpl(u4), tf=7.0, M=1, xnext=mpl(xo))

    # ---- Chebyshev (chebyshev.hpp:113-232) -----------------------------------
    def cheb_points(n):
        return [mp.cos(j * mp.pi / n) for j in range(n + 1)]

    def cheb_D(n):
        xv = cheb_points(n)
        cc = [(2 if j in (0, n) else 1) * (-1) ** j for j in range(n + 1)]
        D = [[mp.mpf(0)] * (n + 1) for _ in range(n + 1)]
        for i in range(n + 1):
            for j in range(n + 1):
                if i != j:
                    D[i][j] = (cc[i] / mp.mpf(cc[j])) / (xv[i] - xv[j])
            D[i][i] = -mp.fsum(D[i][j] for j in range(n + 1) if j != i)
        return D

    def cc_weights(n):
        th = [j * mp.pi / n for j in range(n + 1)]
        w = [mp.mpf(0)] * (n + 1)
        v = [mp.mpf(1)] * (n - 1)
        if n % 2 == 0:
            w[0] = 1 / mp.mpf(n * n - 1); w[n] = w[0]
            for k in range(1, n // 2):
                v = [vi - 2 * mp.cos(2 * k * th[i + 1]) / (4 * k * k - 1) for i, vi in enumerate(v)]
            v = [vi - mp.cos(n * th[i + 1]) / (n * n - 1) for i, vi in enumerate(v)]
        else:
            w[0] = 1 / mp.mpf(n * n); w[n] = w[0]
            for k in range(1, (n - 1) // 2 + 1):
                v = [vi - 2 * mp.cos(2 * k * th[i + 1]) / (4 * k * k - 1) for i, vi in enumerate(v)]
        for i in range(n - 1):
            w[i + 1] = 2 * v[i] / n
        return w

    def comp_D(P, S):
        m, d = S * P + 1, P + 1
        D = cheb_D(P)
        CD = [[mp.mpf(0)] * m for _ in range(m)]
        if S < 2:
            return D
        for i in range(d):
            for j in range(d):
                CD[m - d + i][m - d + j] = D[i][j]
        for k in range(0, (S - 1) * P, P):
            for i in range(P):
                for j in range(d):
                    CD[k + i][k + j] = D[i][j]
        return CD

    cheb = dict(
        points={str(n): mpl(cheb_points(n)) for n in (2, 3, 5, 10)},
        D={str(n): [mpl(r) for r in cheb_D(n)] for n in (2, 3, 5, 10)},
        weights={str(n): mpl(cc_weights(n)) for n in (2, 3, 5, 10)},
        compD={"5x2": [mpl(r) for r in comp_D(5, 2)], "2x3": [mpl(r) for r in comp_D(2, 3)]},
        expansion=dict(coef=[1, 2, 3, 4], x=-1.0, value=-2.0, source="kite_control_test.cpp:205-210"),
        textbook=dict(D2=[[1.5, -2, 0.5], [0.5, 0, -0.5], [-0.5, 2, -1.5]],
                      D5_row0=[8.5, -10.472136, 2.894427, -1.527864, 1.105573, -0.5],
                      w5=[0.04, 0.360743, 0.599257, 0.599257, 0.360743, 0.04],
                      w2=[1 / 3, 4 / 3, 1 / 3], source="Trefethen, Spectral Methods in MATLAB"),
    )

    # ---- path P(theta) (nmpf_node.cpp:30-40) ----------------------------------
    th = sp.symbols("theta", real=True)
    Rr, alt = sp.Rational("2.65"), 0
    qr = [sp.cos(sp.pi / 8), 0, sp.sin(sp.pi / 8), 0]
    Pq = qmul(qmul(qinv(qr), [0, Rr * sp.cos(th), Rr * sp.sin(th), alt]), qr)
    Pv = sp.Matrix(Pq[1:4])
    Pf = sp.lambdify(th, Pv, "mpmath")
    dPf = sp.lambdify(th, Pv.diff(th), "mpmath")
    path = []
    for tv in [-7.0, -2.5, -1.0, 0.0, 0.3, 1.5707963267948966, 2.0, 4.0, 6.5]:
        Pm = Pf(mp.mpf(tv)); dPm = dPf(mp.mpf(tv))
        path.append(dict(theta=tv, P=[float(Pm[i]) for i in range(3)], dP=[float(dPm[i]) for i in range(3)]))

    # ---- collocation residual and cost at the reference test's NLP point ------
    # kite_control_test.cpp:455-526 (full_generics_test): one segment of order
    # 10 on [0, 1], unscaled, path radius 3 rotated by q = (cos pi/24, 0,
    # sin pi/24, 0), Q = 1e-2 diag(1e4, 1e4, 5e3), W = 1e-3, vref = 0.05, no R
    # term, Mayer 2Q on node 0; the 209-vector ARG["x0"] of :582-598.
    # CollocateDynamics (chebyshev.hpp:241-271): G = (CompDiff (x) I15) X -
    # t_scale F(X_i, U_i), t_scale = (tf - t0) / (2 S); CollocateCost (:280-333):
    # Mayer(X_0) + t_scale sum_m w_m L(X_m, U_m).
    fix = json.load(open(os.path.join(HERE, "colloc_full_generics.json")))
    zc = to_mp(fix["z"])
    Pn, Sn = 10, 1
    nn = Pn * Sn + 1
    Xc = [zc[15 * i:15 * i + 15] for i in range(nn)]
    Uc = [zc[15 * nn + 4 * i:15 * nn + 4 * i + 4] for i in range(nn)]
    CDc = comp_D(Pn, Sn)
    tsc = mp.mpf(1) / (2 * Sn)
    Gc = []
    for i in range(nn):
        Fi = aug_f(Xc[i], Uc[i])
        for r in range(15):
            Gc.append(mp.fsum(CDc[i][j] * Xc[j][r] for j in range(nn)) - tsc * Fi[r])
    qc = [sp.cos(sp.pi / 24), 0, sp.sin(sp.pi / 24), 0]
    Pcq = qmul(qmul(qinv(qc), [0, 3 * sp.cos(th), 3 * sp.sin(th), 0]), qc)
    Pcf = sp.lambdify(th, sp.Matrix(Pcq[1:4]), "mpmath")
    Qc = [mp.mpf(100), mp.mpf(100), mp.mpf(50)]
    Wc, vrefc = mp.mpf("0.001"), mp.mpf("0.05")

    def path_res(xv):
        Pm = Pcf(xv[13])
        return [Pm[a] - xv[6 + a] for a in range(3)]

    def lagr(xv):
        rr = path_res(xv)
        return mp.fsum(Qc[a] * rr[a] ** 2 for a in range(3)) + Wc * (vrefc - xv[14]) ** 2

    r0 = path_res(Xc[0])
    mayer = mp.fsum(2 * Qc[a] * r0[a] ** 2 for a in range(3))
    wc = cc_weights(Pn)
    Jc = mayer + tsc * mp.fsum(wc[m] * lagr(Xc[m]) for m in range(nn))
    colloc = dict(source="kite_control_test.cpp:455-598 full_generics_test; chebyshev.hpp:241-333",
                  fixture="colloc_full_generics.json", G=mpl(Gc), J=float(Jc), mayer=float(mayer))

    # ---- the RTI's objective on the shooting grid --------------------------------
    # The reference's Lagrange and Mayer terms (kiteNMPF.cpp:117-141, scaled
    # variables: residual = Sx_r P(theta) - x_r, speed term W (vref_s -
    # x14_s)^2, R u_s^2) with the node's weights, scaling, reference speed and
    # path (kiteNMPF.cpp:32-34, nmpf_node.cpp:30-68), on the build's grid:
    # sum_{k<N} dt L(x_k, u_k) + Mayer(x_N), N = 20, dt = 0.05.
    Qn = [mp.mpf(1000), mp.mpf(1000), mp.mpf(10000)]
    Rn = [mp.mpf("1e-4"), mp.mpf("0.1"), mp.mpf("0.1"), mp.mpf("1e-3")]
    Wn = mp.mpf("1e-3")
    Sxn = [mp.mpf(1) / 10, mp.mpf(1) / 3, mp.mpf(1) / 3, mp.mpf(1) / 2, mp.mpf(1) / 5, mp.mpf(1) / 2,
           mp.mpf(1) / 3, mp.mpf(1) / 3, mp.mpf(1) / 3, 1, 1, 1, 1, 1 / mp.mpf("6.28"), 1 / mp.mpf("6.28")]
    Sun = [1 / mp.mpf("0.15"), 1 / mp.mpf("0.2618"), 1 / mp.mpf("0.2618"), mp.mpf(1) / 5]
    vrefs = Sxn[14] * 4                                    # setReferenceVelocity stores Sx(14,14) v
    Nr, dtr = 20, mp.mpf("0.05")

    def node_res(xv):                                       # scaled path residual, nmpf path
        Pm = Pf(xv[13])
        return [Sxn[6 + a] * Pm[a] - Sxn[6 + a] * xv[6 + a] for a in range(3)]

    rti_cases = []
    rng_c = np.random.default_rng(777)
    for case in range(4):
        Xr = []
        for k in range(Nr + 1):
            xv = np.array(base + [0.0, 0.0], dtype=float)
            xv[0:3] += rng_c.uniform(-1.0, 1.0, 3)
            xv[3:6] += rng_c.uniform(-0.5, 0.5, 3)
            xv[6:9] += rng_c.uniform(-0.3, 0.3, 3)
            xv[9:13] += rng_c.uniform(-0.02, 0.02, 4)
            xv[13] = rng_c.uniform(-3.0, 3.0)
            xv[14] = rng_c.uniform(0.0, 5.0)
            Xr.append([float(t) for t in xv])
        Ur = [[float(rng_c.uniform(0.1, 0.15)), float(rng_c.uniform(-0.12, 0.12)),
               float(rng_c.uniform(-0.12, 0.12)), float(rng_c.uniform(-5, 5))] for _ in range(Nr)]
        Jr = mp.mpf(0)
        for k in range(Nr + 1):
            xv = to_mp(Xr[k])
            rr = node_res(xv)
            Lk = mp.fsum(Qn[a] * rr[a] ** 2 for a in range(3))
            if k == Nr:
                Jr += Lk                                    # Mayer: Q on the path residual only
            else:
                uv = to_mp(Ur[k])
                Lk += Wn * (vrefs - Sxn[14] * xv[14]) ** 2
                Lk += mp.fsum(Rn[j] * (Sun[j] * uv[j]) ** 2 for j in range(4))
                Jr += dtr * Lk
        rti_cases.append(dict(X=Xr, U=Ur, J=float(Jr)))
    rti_cost = dict(source="kiteNMPF.cpp:117-141 terms, nmpf_node.cpp:30-68 values; build grid N=20 dt=0.05",
                    cases=rti_cases)

    out = dict(
        generator="tests/golden/gen_golden.py (sympy %s, mpmath %s, %d digits)" % (sp.__version__, mp.__version__, mp.mp.dps),
        params_file="data/umx_radian.yaml",
        rhs=rhs_cases, rk4=rk4_cases, rk4_reference_call=rk4_ref_call, chebyshev=cheb,
        path=dict(radius=2.65, altitude=0.0, q=[math.cos(math.pi / 8), 0.0, math.sin(math.pi / 8), 0.0], cases=path),
        colloc=colloc, rti_cost=rti_cost,
    )
    with open(os.path.join(HERE, "kite_golden.json"), "w") as fobj:
        json.dump(out, fobj, indent=1)
    print("wrote", os.path.join(HERE, "kite_golden.json"), "rhs", len(rhs_cases), "rk4", len(rk4_cases))


if __name__ == "__main__":
    main()
