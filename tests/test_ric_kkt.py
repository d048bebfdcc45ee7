"""Independent optimality certificate of the multiple-shooting QP (qp_kernel 3,
openkite_amd/csrc/qp_ric.inc; oracle qp_form 1).

The parity tests compare the GPU RTI with the oracle, whose QP solver is the
same Mehrotra method; a flaw shared by both would pass them.  Here the GPU's
QP solution is checked against the first-order conditions of the QP itself,
with no interior-point or Riccati code involved (numpy + scipy NNLS):

  * QP data (scaled A_k, B_k, d_k, residual rows J_k, r_k, control terms,
    bounds) from the oracle's build_msqp at the linearisation point the
    prologue produces (tests/test_gpu_parity.py establishes that the GPU
    linearises identically);
  * the solution read back from the step the GPU applied: dx_k = Sx (X_new -
    X_lin), du_k = Su (U_new - U_lin);
  * dynamics: dx_{k+1} = A_k dx_k + B_k du_k + d_k must hold;
  * condensing in numpy (dx = G w + g, w = [du, dtheta_0, dthetadot_0]) gives
    the gradient of the smooth part (path and speed residuals, R, the
    Levenberg-Marquardt term); the soft state bounds are exact L1 penalties:
    a violated bound contributes soft_weight times its normal, an active one
    a multiplier in [0, soft_weight]; control and theta_0 boxes are hard;
  * multipliers of the (near-)active set by non-negative least squares:
    stationarity residual, feasibility, the multiplier bound and approximate
    complementarity (multiplier x slack of every near-active row) are the KKT
    conditions.
"""
import numpy as np
import pytest

import openkite_amd as ok
from oracle import ffi

M, K = 2, 16
ACT_TOL = 1e-2      # rows with slack below this may carry a multiplier ...
COMP_BAR = 1e-8     # ... as long as multiplier x slack stays below this (relative)
# stationarity bar relative to the gradient scale: the IPM stops on a scaled
# residual < 1e-10 (freeze); at N = 40 the condensed gradient is up to ~1e3 x
# larger than the Riccati-scaled one
STAT_BAR = 1e-7


def condensed_kkt(q, N, dx, du, soft_w, lm):
    """KKT residual of the MS QP at (dx, du) (scaled), relative to the
    gradient scale; also the dynamics residual and the worst hard-bound
    violation."""
    from scipy.optimize import nnls
    nx, nu = 15, 4
    n = nu * N + 2
    # dynamics residual
    dyn = 0.0
    for k in range(N):
        pred = q["A"][k] @ dx[k] + q["B"][k] @ du[k] + q["d"][k]
        dyn = max(dyn, np.abs(pred - dx[k + 1]).max() / max(1.0, np.abs(dx[k + 1]).max()))
    # sensitivities G_k = d dx_k / d w
    G = np.zeros((N + 1, nx, n))
    G[0, 13, nu * N] = 1.0
    G[0, 14, nu * N + 1] = 1.0
    for k in range(N):
        G[k + 1] = q["A"][k] @ G[k]
        G[k + 1][:, nu * k:nu * k + nu] += q["B"][k]
    w = np.concatenate([du.reshape(-1), [dx[0, 13], dx[0, 14]]])
    grad = np.zeros(n)
    for k in range(N + 1):
        nres = 4 if k < N else 3
        Jk = q["J"][k, :nres]
        e = q["r"][k, :nres] + Jk @ dx[k]
        xk = dx[k].copy()
        if k == 0:
            xk[:13] = 0.0                                   # the kite part of node 0 is fixed
        grad += G[k].T @ (Jk.T @ e + lm * xk)
        if k < N:
            grad[nu * k:nu * k + nu] += q["Rh"] * du[k] + q["rho"][k] + lm * du[k]
    # bounds: hard (controls, theta_0), soft (states of nodes 1..N)
    nv = (N + 1) * 19 - 4
    lo, hi = q["lo"], q["hi"]
    cands, hard_viol, scale = [], 0.0, np.abs(grad).max() + 1.0
    g0 = grad.copy()
    for vi in range(nv):
        k, s = divmod(vi, 19)
        if k == 0 and s < 13:
            continue
        if s < 15:
            val, normal, soft = dx[k, s], G[k, s], k > 0
        else:
            val, normal, soft = du[k, s - 15], np.eye(n)[nu * k + s - 15], False
        for bnd, sign in ((lo[vi], 1.0), (hi[vi], -1.0)):
            if not np.isfinite(bnd):
                continue
            slack = sign * (val - bnd)
            if soft and slack < -ACT_TOL * max(1.0, abs(bnd)):
                g0 -= soft_w * sign * normal                 # violated: the penalty's full weight
            else:
                cands.append((sign * normal, soft, max(slack, 0.0) / max(1.0, abs(bnd))))
            if not soft:
                hard_viol = max(hard_viol, -slack)
    # near-active rows by growing slack tolerance: the first set whose NNLS
    # multipliers meet stationarity AND approximate complementarity (an
    # interior-point solution holds weakly active rows at slack ~ mu / z)
    results = [(np.abs(g0).max(), not cands, 0)]
    for tol in (1e-8, 1e-6, 1e-5, 1e-4, 1e-3, ACT_TOL):
        rows = [c for c in cands if c[2] <= tol]
        if not rows:
            continue
        A = np.array([r for r, _, _ in rows])
        lam, _ = nnls(A.T, g0, maxiter=50 * n)
        st = np.abs(g0 - A.T @ lam).max()
        soft_mask = np.array([sf for _, sf, _ in rows])
        comp = float(np.max(lam * np.array([sl for _, _, sl in rows]))) / scale
        ok = bool(np.all(lam[soft_mask] <= soft_w * (1 + 1e-6))) and comp < COMP_BAR
        results.append((st, ok, len(rows)))
        if ok and st / scale < 1e-9:
            break
    good = [r for r in results if r[1]]
    best = min(good or results, key=lambda r: r[0])
    stat, mult_ok, nrows = best
    return stat / scale, dyn, hard_viol, mult_ok, nrows


def _cfg(N):
    c = ffi.node_config(N=N)
    return c, ffi.cfg_vector(c)


def test_certificate_on_oracle_ms_qp(kp):
    """The certificate (CPU) accepts the oracle's multiple-shooting QP solutions
    over 3 closed-loop steps at N = 20 and 40, and rejects a perturbed one."""
    for N in (20, 40):
        c, cv = _cfg(N)
        B = 3
        xs = ffi.synthetic_states(B, offset=8100)
        x = np.zeros((B, 15)); x[:, :13] = xs
        for b in range(B):
            x[b, 13] = ffi.closest_point(cv, xs[b, 6:9])
        X, U = np.zeros((B, N + 1, 15)), np.zeros((B, N, 4))
        Sx, Su = np.array(c["Sx"]), np.array(c["Su"])
        for step in range(3):
            for b in range(B):
                _, Xl, Ul, _ = ffi.prologue(kp, cv, N, M, x[b], X[b], U[b], warm=int(step > 0))
                q = ffi.msqp_build(kp, cv, N, M, Xl, Ul)
                v, kkt, _ = ffi.msqp_solve(kp, cv, N, M, Xl, Ul, K)
                assert kkt < 1e-8
                dx = np.array([v[k * 19:k * 19 + 15] for k in range(N + 1)])
                du = np.array([v[k * 19 + 15:k * 19 + 19] for k in range(N)])
                stat, dyn, hv, mok, nact = condensed_kkt(q, N, dx, du, c["soft_weight"], c["lm"])
                assert stat < STAT_BAR and dyn < 1e-9 and hv < 1e-9 and mok, (N, step, b, stat, dyn, hv, nact)
                if step == 0 and b == 0:
                    du2 = du.copy(); du2[2, 1] += 1e-3
                    dx2 = dx.copy()
                    for k in range(N):
                        dx2[k + 1] = q["A"][k] @ dx2[k] + q["B"][k] @ du2[k] + q["d"][k]
                    assert condensed_kkt(q, N, dx2, du2, c["soft_weight"], c["lm"])[0] > 100 * STAT_BAR
            ffi.rti_step(kp, cv, N, M, K, x, X, U, warm=int(step > 0))
            x = X[:, 1, :].copy()


@pytest.mark.gpu
@pytest.mark.parametrize("N,mode", [(20, "default"), (40, "default"), (20, "every_node")])
def test_gpu_ric_solution_satisfies_kkt(kp, N, mode):
    """The GPU's multiple-shooting QP solutions (k_qp_ric) over 4 closed-loop
    steps of 16 kites satisfy the QP's KKT conditions: stationarity <= 1e-6
    relative (QPs that stopped at the cap K: 1e-4), dynamics and hard bounds to
    1e-9, soft-bound multipliers within [0, soft_weight].  `every_node`: the
    undamped exact-bound configuration (qp_lm 0, soft weight 1e6)
    with a binding |omega_i| <= 3 box."""
    B = 16
    c, cv = _cfg(N)
    cfg = ok.default_config(N=N, qp_kernel=3)
    if mode == "every_node":
        c["lm"], c["soft_weight"] = 0.0, 1e6
        c["lbx"][3:6] = [-3.0] * 3
        c["ubx"][3:6] = [3.0] * 3
        cv = ffi.cfg_vector(c)
        cfg.qp_lm, cfg.qp_soft_weight = 0.0, 1e6
        for i in range(3, 6):
            cfg.lbx[i], cfg.ubx[i] = -3.0, 3.0
    xs = ffi.synthetic_states(B, offset=8200)
    x = np.zeros((B, 15)); x[:, :13] = xs
    for b in range(B):
        x[b, 13] = ffi.closest_point(cv, xs[b, 6:9])
    Sx, Su = np.array(c["Sx"]), np.array(c["Su"])
    g = ok.BatchNMPC(ok.load_properties(), cfg, B)
    checked, worst = 0, 0.0
    try:
        Xp, Up = np.zeros((B, N + 1, 15)), np.zeros((B, N, 4))
        for step in range(4):
            r = g.step(x)
            for b in range(B):
                if r["status"][b] & 32:
                    continue
                _, Xl, Ul, _ = ffi.prologue(kp, cv, N, M, x[b], Xp[b], Up[b], warm=int(step > 0))
                q = ffi.msqp_build(kp, cv, N, M, Xl, Ul)
                dx = (r["traj"][b] - Xl) * Sx
                du = (r["ctrl"][b] - Ul) * Su
                stat, dyn, hv, mok, nact = condensed_kkt(q, N, dx, du, c["soft_weight"], c["lm"])
                bar = 1e-4 if r["status"][b] & 2 else STAT_BAR
                assert stat < bar and dyn < 1e-9 and hv < 1e-9 and mok, (step, b, stat, dyn, hv, nact)
                worst = max(worst, stat)
                checked += 1
            Xp, Up = r["traj"].copy(), r["ctrl"].copy()
            x = r["traj"][:, 1, :].copy()
    finally:
        g.close()
    assert checked >= 3 * B
    print(f"N={N} {mode}: {checked} GPU multiple-shooting QP solutions, stationarity <= {worst:.1e}")
