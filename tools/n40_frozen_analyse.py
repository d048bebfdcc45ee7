"""Analysis of tools/n40_frozen_dump.py, CPU only.

For every step and kite of the N = 40 condensed-QP test sequence:
  * e_plan  : GPU plan vs oracle plan (the test's per-kite error)
  * dH, dh  : GPU QP data vs the oracle's (same linearisation point), relative
  * s_solve : the ORACLE's IPM on the GPU's own QP data vs the GPU's plan --
              solver parity with the data held equal
  * s_data  : the oracle's IPM on the GPU's data vs on its own data -- the
              plan's sensitivity to the actual GPU/oracle data difference
  * s_1e15  : the oracle's plan under a 1e-15 relative symmetric perturbation
              of H (the envelope probe of tests/test_oracle.py)
  * s_meas  : the same at the measured relative size of H_gpu - H_orc
plus the cost, KKT residual and reduced-Hessian picture for the worst kite.
  python tools/n40_frozen_analyse.py DUMPDIR [qk ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from oracle import ffi  # noqa: E402
from test_gpu_parity import condensed_cfgv, gpu_to_oracle_perm  # noqa: E402

Nh, M, K = 40, 2, 16
kp = ffi.load_params()
cv = condensed_cfgv(Nh)
perm = gpu_to_oracle_perm(Nh)
n = 4 * Nh + 2


def plan_of(q, Xp, Up, w):
    """Plan (traj, ctrl) of scaled step w at the linearisation point, as the
    oracle's expansion: dx = G D w (G from build_qp), du = D w."""
    dw = q["D"] * w
    traj = Xp + q["g"] + np.einsum("kin,n->ki", q["G"], dw)
    ctrl = Up + dw[:4 * Nh].reshape(Nh, 4)
    return traj, ctrl


def rel(a, b):
    return np.abs(a - b).max() / max(1.0, np.abs(b).max())


def cost(H, h, w):
    return 0.5 * w @ H @ w + h @ w


def main(d, qks):
    for qk in qks:
        z = np.load(os.path.join(d, f"n40_frozen_qk{qk}.npz"))
        S, B = z["kkt_g"].shape
        print(f"=== qp_kernel {qk}: {S} steps x {B} kites")
        print(" st  k  e_plan    kkt_g    kkt_o    it_g it_o dH       dh       dC       s_solve  s_data   s_1e15   "
              "s_meas   kkt_og   e_capped")
        worst = None
        for s in range(S):
            for b in range(B):
                e_plan = max(rel(z["traj_g"][s, b], z["traj_o"][s, b]), rel(z["ctrl_g"][s, b], z["ctrl_o"][s, b]))
                st, Xp, Up, _ = ffi.prologue(kp, cv, Nh, M, z["x"][s, b], z["Xin"][s, b], z["Uin"][s, b],
                                             warm=int(s > 0))
                q = ffi.build_qp(kp, cv, Nh, M, Xp, Up, want_G=True)
                Hg = np.zeros((n, n)); Hg[np.ix_(perm, perm)] = z["H"][s, b]
                hg = np.zeros(n); hg[perm] = z["h"][s, b]
                Cg = np.zeros((Nh, n)); Cg[:, perm] = z["C"][s, b]
                dH = np.abs(Hg - q["H"]).max() / np.abs(q["H"]).max()
                dh = np.abs(hg - q["h"]).max() / max(1.0, np.abs(q["h"]).max())
                dC = np.abs(Cg[:q["m"]] - q["C"]).max() / max(1.0, np.abs(q["C"]).max()) if q["m"] else 0.0
                wo, ko = ffi.qp_solve(q["H"], q["h"], q["lb"], q["ub"], q["C"], q["c"], K)
                wg, kg = ffi.qp_solve(Hg, hg, q["lb"], q["ub"], Cg[:q["m"]], q["c"], K)
                to, uo = plan_of(q, Xp, Up, wo)
                tg, ug = plan_of(q, Xp, Up, wg)
                s_solve = max(rel(z["traj_g"][s, b], tg), rel(z["ctrl_g"][s, b], ug))
                s_data = max(rel(tg, to), rel(ug, uo))
                E = np.random.default_rng(1000 * b + s).normal(size=(n, n))
                E = (E + E.T) / 2
                w1, k1 = ffi.qp_solve(q["H"] * (1 + 1e-15 * E), q["h"], q["lb"], q["ub"], q["C"], q["c"], K)
                t1, u1 = plan_of(q, Xp, Up, w1)
                w2, k2 = ffi.qp_solve(q["H"] * (1 + dH * E), q["h"], q["lb"], q["ub"], q["C"], q["c"], K)
                t2, u2 = plan_of(q, Xp, Up, w2)
                s15 = max(rel(t1, to), rel(u1, uo)) if k1 < 1e-10 and ko < 1e-10 else np.nan
                sm = max(rel(t2, to), rel(u2, uo)) if k2 < 1e-10 and ko < 1e-10 else np.nan
                # the oracle's own RTI step on this kite, its iteration count, and
                # the same step with the IPM capped at the GPU's iteration count
                def orc(Kc):
                    X1, U1 = z["Xin"][s, b][None].copy(), z["Uin"][s, b][None].copy()
                    its = np.zeros(1, dtype=np.int32)
                    ffi.rti_step(kp, cv, Nh, M, Kc, z["x"][s, b][None].copy(), X1, U1, warm=int(s > 0), iters=its)
                    return X1[0], U1[0], int(its[0])
                _, _, it_o = orc(K)
                it_g = int(z["it_g"][s, b])
                Xc, Uc, _ = orc(it_g) if it_g > 0 else (None, None, 0)
                e_cap = max(rel(z["traj_g"][s, b], Xc), rel(z["ctrl_g"][s, b], Uc)) if it_g > 0 else np.nan
                print(f" {s}  {b:2d} {e_plan:8.1e} {z['kkt_g'][s, b]:8.1e} {z['diag_o'][s, b, 5]:8.1e} {it_g:4d} "
                      f"{it_o:4d} {dH:8.1e} {dh:8.1e} {dC:8.1e} {s_solve:8.1e} {s_data:8.1e} {s15:8.1e} {sm:8.1e} "
                      f"{kg:8.1e} {e_cap:8.1e}")
                if worst is None or e_plan > worst[0]:
                    worst = (e_plan, s, b, q, Hg, hg, Cg, wo, wg, Xp, Up)
        e_plan, s, b, q, Hg, hg, Cg, wo, wg, Xp, Up = worst
        print(f"--- worst kite: step {s} kite {b}, plan error {e_plan:.2e}")
        # the GPU's scaled step, recovered from its plan (du = D w on the controls,
        # dtheta0 / dthetadot0 = D w on the last two variables)
        Dv = q["D"]
        wgpu = np.concatenate([(z["ctrl_g"][s, b] - Up).reshape(-1), z["traj_g"][s, b][0, 13:15] - Xp[0, 13:15]]) / Dv
        rd_o = q["H"] @ wo + q["h"]
        rd_g = q["H"] @ wgpu + q["h"]
        print(f"  GPU step vs oracle step: |w_gpu - w_oo|_inf {np.abs(wgpu - wo).max():.2e}; max|H| "
              f"{np.abs(q['H']).max():.2e} (freeze test scales the dual residual by 1/(1 + max|H|))")
        print(f"  cost at w_oo {cost(q['H'], q['h'], wo):.12e}, at w_gpu {cost(q['H'], q['h'], wgpu):.12e}")
        # a third fp64 implementation of the same IPM, differing only in its
        # rounding (numpy replica of qp_ipm, LAPACK Cholesky, same z0 / freeze)
        from warm_ipm_probe import ipm
        wn, _, _, itn, rn = ipm(q, K, z_init=20.0)
        print(f"  numpy/LAPACK replica: {itn} iterations, residual {rn:.1e}, |w_np - w_oo|_inf "
              f"{np.abs(wn - wo).max():.2e}, |w_np - w_gpu|_inf {np.abs(wn - wgpu).max():.2e}")
        dw = wgpu - wo
        print(f"  Rayleigh quotient of w_gpu - w_oo: {dw @ q['H'] @ dw / (dw @ dw):.2e} (max|H| "
              f"{np.abs(q['H']).max():.2e}); of w_np - w_oo: "
              f"{(wn - wo) @ q['H'] @ (wn - wo) / max((wn - wo) @ (wn - wo), 1e-300):.2e}")
        print(f"  |w_og - w_oo|_inf {np.abs(dw).max():.2e}; cost(H_o) at w_oo {cost(q['H'], q['h'], wo):.12e}, "
              f"at w_og {cost(q['H'], q['h'], wg):.12e}")
        # active set at the oracle solution and the reduced Hessian on its null space
        tol = 1e-7
        act_lo = np.where(wo - q["lb"] < tol * np.maximum(1, np.abs(q["lb"])))[0]
        act_hi = np.where(q["ub"] - wo < tol * np.maximum(1, np.abs(q["ub"])))[0]
        Cw = q["C"] @ wo if q["m"] else np.zeros(0)
        act_c = np.where(Cw - q["c"] < tol * np.maximum(1, np.abs(q["c"])))[0] if q["m"] else np.zeros(0, int)
        A = np.zeros((len(act_lo) + len(act_hi) + len(act_c), n))
        r = 0
        for i in list(act_lo) + list(act_hi):
            A[r, i] = 1.0; r += 1
        for k in act_c:
            A[r] = q["C"][k]; r += 1
        print(f"  active: {len(act_lo)} lower, {len(act_hi)} upper, {len(act_c)} vx rows of {q['m']}")
        if A.shape[0]:
            _, sv, Vt = np.linalg.svd(A)
            Z = Vt[np.sum(sv > 1e-12):].T
        else:
            Z = np.eye(n)
        Hr = Z.T @ q["H"] @ Z
        ev = np.linalg.eigvalsh(Hr)
        print(f"  reduced Hessian: dim {Hr.shape[0]}, eigenvalues min {ev[0]:.2e} max {ev[-1]:.2e} "
              f"cond {ev[-1] / max(ev[0], 1e-300):.2e}")
        dz = Z.T @ dw
        print(f"  share of dw in the free subspace {np.linalg.norm(Z @ dz) / max(np.linalg.norm(dw), 1e-300):.3f}")
        if Hr.shape[0]:
            lam, U = np.linalg.eigh(Hr)
            c = U.T @ dz
            wgt = c ** 2 / max((c ** 2).sum(), 1e-300)
            top = np.argsort(wgt)[::-1][:5]
            print("  dw along reduced-Hessian eigenvectors: " +
                  ", ".join(f"lambda {lam[i]:.1e}: {wgt[i]:.3f}" for i in top))


if __name__ == "__main__":
    main(sys.argv[1], [int(a) for a in sys.argv[2:]] or [1, 2])
