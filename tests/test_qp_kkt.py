"""Independent optimality certificate for the GPU QP solutions.

The parity tests compare the GPU RTI with the oracle, whose QP is the same
Mehrotra interior-point method; a flaw shared by both would pass them.  This
file checks the GPU solution against the first-order (KKT) conditions of the
QP the GPU itself condensed, with no interior-point code involved:

  min 1/2 w'Hw + h'w   s.t.  lb <= w <= ub,  C w >= c        (scaled variables)

* H, h, C, c come from kite_nmpc_get_qp (the GPU condensing);
* w is read back from the step the GPU applied: du = U_new - U_lin,
  dtheta0/dthetadot0 from the first trajectory node, w = du / D with
  D = 1/Su (controls), 1/Sx13, 1/Sx14 (theta0, thetadot0);
* the active set is {constraints with slack <= 1e-6 * max(1, |bound|)} and
  the multipliers are the non-negative least-squares fit of H w + h onto the
  active constraint normals (scipy.optimize.nnls): stationarity residual,
  primal feasibility and dual sign (lambda >= 0 by construction) together
  are the KKT conditions.

Prototype on oracle QPs: stationarity ~1e-14 relative at active-set tolerance
1e-6.  Bar here: stationarity and feasibility <= 1e-8 relative to
max|H| max|w| + max|h| (the GPU IPM freezes at a 1e-10 KKT residual); QPs
that hit the iteration cap K = 16 (status bit 2: at N = 40 several do on the
third closed-loop step, oracle and GPU alike, with identical certificates)
are held to 1e-6, the residual below which the RTI accepts the step.
"""
import numpy as np
import pytest

import openkite_amd as ok
from oracle import ffi

M, K = 2, 16
ACT_TOL = 1e-6
KKT_TOL = 1e-8
KKT_TOL_CAPPED = 1e-6     # QPs stopped by the iteration cap (status bit 2) whose step was still
                          # accepted (IPM residual < 1e-6, the step safeguard's bar)


def gpu_perm(N):
    """GPU QP column j -> oracle column (oracle: [u_k(4)]_k, theta0, thetadot0)."""
    p = []
    for j in range(4 * N + 2):
        if j < 3 * N:
            p.append(4 * (j // 3) + j % 3)
        elif j < 4 * N:
            p.append(4 * (j - 3 * N) + 3)
        else:
            p.append(j)
    return np.array(p)


def kkt_certificate(H, h, lb, ub, C, c, w, extra=None):
    """extra: (A, s, bnd) further constraints A w >= ... with slacks s (the state
    bounds the lazy rows enforce; bnd: the bound each slack refers to)."""
    from scipy.optimize import nnls
    n = w.size
    g = H @ w + h
    sl, su, sc = w - lb, ub - w, C @ w - c
    rows = []
    if extra is not None:
        for a, s_, bd in zip(*extra):
            if s_ <= ACT_TOL * max(1.0, abs(bd)):
                rows.append(a)
    for i in range(n):
        if sl[i] <= ACT_TOL * max(1.0, abs(lb[i])):
            e = np.zeros(n); e[i] = 1.0; rows.append(e)
        if su[i] <= ACT_TOL * max(1.0, abs(ub[i])):
            e = np.zeros(n); e[i] = -1.0; rows.append(e)
    for r in range(c.size):
        if sc[r] <= ACT_TOL * max(1.0, abs(c[r])):
            rows.append(C[r])
    scale = np.abs(H).max() * max(1e-300, np.abs(w).max()) + np.abs(h).max()
    if rows:
        A = np.array(rows)
        lam, _ = nnls(A.T, g, maxiter=50 * n)
        res = g - A.T @ lam
    else:
        res = g
    feas = max(0.0, -sl.min(), -su.min(), -(sc.min() if c.size else 0.0))
    return np.abs(res).max() / scale, feas / scale, len(rows)


def scaled_solution(cfg, N, U_lin, X_lin, U_new, X_new):
    Su = np.array(cfg.Su)
    du = (U_new - U_lin) * Su                         # w = du / D, D = 1/Su
    w_or = np.zeros(4 * N + 2)
    w_or[:4 * N] = du.reshape(-1)
    w_or[4 * N] = (X_new[0, 13] - X_lin[0, 13]) * cfg.Sx[13]
    w_or[4 * N + 1] = (X_new[0, 14] - X_lin[0, 14]) * cfg.Sx[14]
    lb = np.zeros(4 * N + 2); ub = np.zeros(4 * N + 2)
    lb[:4 * N] = ((np.array(cfg.lbu) - U_lin) * Su).reshape(-1)
    ub[:4 * N] = ((np.array(cfg.ubu) - U_lin) * Su).reshape(-1)
    lb[4 * N], ub[4 * N] = -cfg.theta_flex * cfg.Sx[13], cfg.theta_flex * cfg.Sx[13]
    lb[4 * N + 1], ub[4 * N + 1] = -cfg.theta_flex * cfg.Sx[14], cfg.theta_flex * cfg.Sx[14]
    p = gpu_perm(N)
    return w_or[p], lb[p], ub[p]


def state_bound_rows(q_or, cfg, N, X_new):
    """Finite bounds of states 1..12 at nodes 1..N as constraints on the scaled
    GPU variables: +-G_k[i] D w >= ..., slacks from the trajectory the GPU
    applied (the expansion is linear in w, so X_new = x(w) exactly)."""
    p = gpu_perm(N)
    A, s, bnd = [], [], []
    for k in range(1, N + 1):
        for i in range(1, 13):
            row = (q_or["G"][k, i] * q_or["D"])[p]
            lo, hi = cfg.lbx[i], cfg.ubx[i]
            if np.isfinite(lo):
                A.append(row); s.append(X_new[k, i] - lo); bnd.append(lo)
            if np.isfinite(hi):
                A.append(-row); s.append(hi - X_new[k, i]); bnd.append(hi)
    return np.array(A), np.array(s), np.array(bnd)


def test_certificate_on_oracle_closed_loop(kp):
    """The certificate itself (CPU): it accepts the oracle's IPM solutions along
    3 closed-loop steps and rejects a perturbed solution."""
    N = 20
    cfg = ok.default_config(N=N, qp_kernel=2)
    cv = ffi.cfg_vector(dict(ffi.node_config(N=N), qp_form=0))
    B = 4
    xs = ffi.synthetic_states(B, offset=8000)
    x = np.zeros((B, 15)); x[:, :13] = xs
    for b in range(B):
        x[b, 13] = ffi.closest_point(cv, xs[b, 6:9])
    X, U = np.zeros((B, N + 1, 15)), np.zeros((B, N, 4))
    inv = np.argsort(gpu_perm(N))
    for step in range(3):
        Xp, Up = X.copy(), U.copy()
        ffi.rti_step(kp, cv, N, M, K, x, X, U, warm=int(step > 0))
        for b in range(B):
            _, Xl, Ul, _ = ffi.prologue(kp, cv, N, M, x[b], Xp[b], Up[b], warm=int(step > 0))
            q = ffi.build_qp(kp, cv, N, M, Xl, Ul)
            w, lb, ub = (a[inv] for a in scaled_solution(cfg, N, Ul, Xl, U[b], X[b]))
            np.testing.assert_allclose(lb, q["lb"], atol=1e-14)
            np.testing.assert_allclose(ub, q["ub"], atol=1e-14)
            stat, feas, _ = kkt_certificate(q["H"], q["h"], lb, ub, q["C"], q["c"], w)
            assert stat < KKT_TOL and feas < KKT_TOL, (step, b, stat, feas)
            # a solution moved off the optimum along a free direction fails
            free = np.where((w - lb > 1e-3) & (ub - w > 1e-3))[0]
            if free.size:
                w2 = w.copy(); w2[free[0]] += 1e-3 * (ub[free[0]] - lb[free[0]])
                assert kkt_certificate(q["H"], q["h"], lb, ub, q["C"], q["c"], w2)[0] > 1e3 * KKT_TOL
        x = X[:, 1, :].copy()


@pytest.mark.gpu
@pytest.mark.parametrize("N,qp_kernel", [(20, 2), (20, 1), (40, 2)])
def test_gpu_qp_solution_satisfies_kkt(kp, N, qp_kernel):
    B = 16
    cfg = ok.default_config(N=N, qp_kernel=qp_kernel)
    cv = ffi.cfg_vector(dict(ffi.node_config(N=N), qp_form=0))
    xs = ffi.synthetic_states(B, offset=8000)
    x = np.zeros((B, 15)); x[:, :13] = xs
    for b in range(B):
        x[b, 13] = ffi.closest_point(cv, xs[b, 6:9])
    g = ok.BatchNMPC(ok.load_properties(), cfg, B)
    checked, capped, worst_stat, worst_feas = 0, 0, 0.0, 0.0
    try:
        Xprev, Uprev = np.zeros((B, N + 1, 15)), np.zeros((B, N, 4))
        for step in range(3):
            r = g.step(x)
            for b in range(B):
                if r["status"][b] & 32:          # step rejected: no QP step applied
                    continue
                # linearisation point = the prologue's output (shift / cold start)
                _, Xl, Ul, _ = ffi.prologue(kp, cv, N, M, x[b], Xprev[b], Uprev[b], warm=int(step > 0))
                q = g.get_qp(b)
                w, lb, ub = scaled_solution(cfg, N, Ul, Xl, r["ctrl"][b], r["traj"][b])
                # state bounds (lazy rows; at N = 40 the |q_i| <= 1.01 bound binds on the
                # cold step): their multipliers enter stationarity, their slacks must be >= 0
                A, sx, bnd = state_bound_rows(ffi.build_qp(kp, cv, N, M, Xl, Ul, want_G=True), cfg, N,
                                              r["traj"][b])
                if not r["status"][b] & 8:
                    assert sx.min() >= -1e-8 * np.abs(bnd).max(), (step, b, sx.min())
                stat, feas, nact = kkt_certificate(q["H"], q["h"], lb, ub, q["C"], q["cl"], w, (A, sx, bnd))
                worst_stat, worst_feas = max(worst_stat, stat), max(worst_feas, feas)
                bar = KKT_TOL_CAPPED if r["status"][b] & 2 else KKT_TOL
                capped += int(r["status"][b] & 2 != 0)
                assert stat < bar and feas < bar, (step, b, stat, feas, nact, r["status"][b])
                checked += 1
            Xprev, Uprev = r["traj"].copy(), r["ctrl"].copy()
            x = r["traj"][:, 1, :].copy()
    finally:
        g.close()
    assert checked >= 2 * B
    print(f"N={N} qp_kernel={qp_kernel}: {checked} GPU QP solutions ({capped} stopped by the iteration cap), "
          f"KKT stationarity <= {worst_stat:.1e}, feasibility <= {worst_feas:.1e}")
