"""Warm-start study for the condensed N = 20 QP: the
oracle closed loop (bench workload, B kites) generates the QPs; a numpy replica
of the oracle IPM (oracle/kite_oracle.cpp qp_ipm) solves each one cold and from
the previous step's shifted slacks / multipliers.  Tools only (loads the
oracle).
  python tools/warm_ipm_probe.py [B] [STEPS]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle import ffi  # noqa: E402

FREEZE, TAU0 = 1e-10, 0.995


def ipm(q, K, w0=None, s0=None, z0=None, s_floor=0.1, z_init=10.0):
    H, h, lb, ub, C, c = q["H"], q["h"], q["lb"], q["ub"], q["C"], q["c"]
    n, m = H.shape[0], C.shape[0]
    A = np.vstack([np.eye(n), -np.eye(n), C])
    b = np.concatenate([lb, -ub, c])
    if w0 is None:
        mar = 0.1 * (ub - lb)
        w = np.clip(np.zeros(n), lb + mar, ub - mar)
    else:
        w = w0.copy()
    s = np.maximum(A @ w - b, s_floor) if s0 is None else s0.copy()
    z = np.full(A.shape[0], z_init) if z0 is None else z0.copy()
    dsc = 1.0 / (1.0 + np.abs(H).max())
    for it in range(K):
        rp = A @ w - b - s
        rd = H @ w + h - A.T @ z
        mu = s @ z / len(s)
        r = max(np.abs(rp).max(), np.abs(rd).max() * dsc, mu)
        if r < FREEZE or not np.isfinite(r):
            return w, s, z, it, r
        sig = z / s
        Mx = H + A.T @ (sig[:, None] * A)
        L = np.linalg.cholesky(Mx)

        def solve(rc):
            t = rc / s - sig * rp
            dw = np.linalg.solve(L.T, np.linalg.solve(L, -rd + A.T @ t))
            ds = A @ dw + rp
            dz = (rc - z * ds) / s
            return dw, ds, dz

        def mstep(ds, dz):
            a = 1.0
            neg = ds < 0
            if neg.any():
                a = min(a, (-s[neg] / ds[neg]).min())
            neg = dz < 0
            if neg.any():
                a = min(a, (-z[neg] / dz[neg]).min())
            return a
        dwa, dsa, dza = solve(-s * z)
        aa = mstep(dsa, dza)
        mua = (s + aa * dsa) @ (z + aa * dza) / len(s)
        sigma = (mua / mu) ** 3
        dw, ds, dz = solve(-s * z - dsa * dza + sigma * mu)
        tau = max(TAU0, 1.0 - mu)
        a = min(1.0, tau * mstep(ds, dz))
        w += a * dw; s += a * ds; z += a * dz
    rp = A @ w - b - s
    rd = H @ w + h - A.T @ z
    return w, s, z, K, max(np.abs(rp).max(), np.abs(rd).max() * dsc, s @ z / len(s))


def shift_rows(v, n, N, m):
    """Shift a row-indexed vector [box lo (n) | box hi (n) | C rows (m)] by one
    interval: control k <- k + 1 (last kept), theta rows kept, node rows k <- k + 1."""
    out = v.copy()
    for part in (0, n):
        blk = v[part:part + 4 * N].reshape(N, 4)
        out[part:part + 4 * N] = np.vstack([blk[1:], blk[-1:]]).reshape(-1)
    if m:
        per = m // N
        blk = v[2 * n:].reshape(N, per)
        out[2 * n:] = np.vstack([blk[1:], blk[-1:]]).reshape(-1)
    return out


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    N, M, K = 20, 2, 16
    kp = ffi.load_params()
    cfgv = ffi.cfg_vector(ffi.node_config(N=N))
    xs = ffi.synthetic_states(B)
    x0 = np.zeros((B, 15)); x0[:, :13] = xs
    for b in range(B):
        x0[b, 13] = ffi.closest_point(cfgv, xs[b, 6:9])
    X = np.zeros((B, N + 1, 15)); U = np.zeros((B, N, 4))
    variants = {"cold": {}, "warm_z": dict(zfloor=1e-2, sfloor=1e-2), "warm_z3": dict(zfloor=1e-3, sfloor=1e-3),
                "warm_mu": dict(mu0=1e-2), "warm_mu3": dict(mu0=1e-3), "warm_mu4": dict(mu0=1e-4)}
    its = {k: [] for k in variants}
    errs = {k: [] for k in variants}
    prev = [None] * B
    for st in range(STEPS):
        warm = 1 if st else 0
        oit = np.zeros(B, dtype=np.int32)
        qps = []
        for b in range(B):
            _, Xp, Up, _ = ffi.prologue(kp, cfgv, N, M, x0[b], X[b], U[b], warm)
            qps.append(ffi.build_qp(kp, cfgv, N, M, Xp, Up))
        u0, diag, status = ffi.rti_step(kp, cfgv, N, M, K, x0, X, U, warm, iters=oit)
        for b in range(B):
            q = qps[b]
            n, m = q["H"].shape[0], q["m"]
            wc, sc, zc, itc, rc = ipm(q, 40)
            for name, opt in variants.items():
                if name == "cold" or prev[b] is None or prev[b][1].shape[0] != 2 * n + m:
                    w, s, z, it, r = wc, sc, zc, itc, rc
                else:
                    A = np.vstack([np.eye(n), -np.eye(n), q["C"]])
                    bb = np.concatenate([q["lb"], -q["ub"], q["c"]])
                    mar = 0.1 * (q["ub"] - q["lb"])
                    w0 = np.clip(np.zeros(n), q["lb"] + mar, q["ub"] - mar)
                    zp = shift_rows(prev[b][2], n, N, m)
                    sl = A @ w0 - bb
                    if "mu0" in opt:
                        mu0 = opt["mu0"]
                        s0 = np.maximum(sl, np.sqrt(mu0))
                        z0 = np.maximum(zp, mu0 / s0)
                    else:
                        s0 = np.maximum(sl, opt["sfloor"])
                        z0 = np.maximum(zp, opt["zfloor"])
                    w, s, z, it, r = ipm(q, 40, w0=w0, s0=s0, z0=z0)
                its[name].append(it)
                errs[name].append(np.abs(w - wc).max() / max(1.0, np.abs(wc).max()))
            if itc != oit[b] and oit[b] < K:
                print(f"step {st} kite {b}: replica {itc} vs oracle {oit[b]} iterations")
            prev[b] = (wc, sc, zc)
        x0 = np.zeros((B, 15))
        x0[:] = X[:, 1, :] if False else X[:, 0, :]
        # bench closed loop: the next measured state is the predicted node 1
        x0 = X[:, 1, :].copy()
        print(f"step {st:2d}: " + "  ".join(f"{k} {np.mean(its[k][-B:]):5.2f}" for k in variants), flush=True)
    for k in variants:
        a = np.array(its[k][B:]); e = np.array(errs[k][B:])
        print(f"{k:10s} mean {a.mean():6.2f} p90 {np.percentile(a, 90):5.1f} max {a.max():3d}  "
              f">=16: {np.mean(a >= 16):.3f}  sol err max {e.max():.2e}")


if __name__ == "__main__":
    main()
