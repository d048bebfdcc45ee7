"""Active-set study for the condensed N = 20 QP:
along the oracle closed loop (bench workload), the size of the active set at
the IPM solution, its change against the previous step's shifted active set,
and the iterations a primal-dual active-set method (Hintermueller-Ito-Kunisch,
box constraints only) needs from that warm start and from a cold start.
Tools only (loads the oracle).   python tools/active_set_probe.py"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tools"))
from oracle import ffi
from warm_ipm_probe import ipm
B, STEPS, N, M, K = 32, 12, 20, 2, 16
kp = ffi.load_params(); cfgv = ffi.cfg_vector(ffi.node_config(N=N))
xs = ffi.synthetic_states(B); x0 = np.zeros((B, 15)); x0[:, :13] = xs
for b in range(B): x0[b, 13] = ffi.closest_point(cfgv, xs[b, 6:9])
X = np.zeros((B, N + 1, 15)); U = np.zeros((B, N, 4))
prevA = [None]*B
def pdas(q, Al, Au, maxit=20, cpar=1.0):
    H,h,lb,ub = q["H"],q["h"],q["lb"],q["ub"]; n=len(h)
    hist=[]
    for it in range(maxit):
        F = ~(Al|Au)
        w = np.where(Al, lb, np.where(Au, ub, 0.0))
        rhs = -(h[F] + H[np.ix_(F, ~F)] @ w[~F])
        w[F] = np.linalg.solve(H[np.ix_(F,F)], rhs)
        mu = H@w + h; mu[F]=0
        d = np.diag(H)
        nAl = (mu - cpar*d*(w-lb)) > 0
        nAu = (-mu - cpar*d*(ub-w)) > 0
        if (nAl==Al).all() and (nAu==Au).all():
            return w, it+1, True
        Al, Au = nAl, nAu & ~nAl
    return w, maxit, False
stats=[]
for st in range(STEPS):
    warm = 1 if st else 0
    for b in range(B):
        _, Xp, Up, _ = ffi.prologue(kp, cfgv, N, M, x0[b], X[b], U[b], warm)
        q = ffi.build_qp(kp, cfgv, N, M, Xp, Up)
        n=len(q["h"]); m=q["m"]
        w, s, z, it, r = ipm(q, 40)
        tol=1e-6
        Al = (w-q["lb"]) < tol*(1+np.abs(q["lb"])); Au = (q["ub"]-w) < tol*(1+np.abs(q["ub"]))
        Cact = (q["C"]@w - q["c"]) < 1e-6 if m else np.zeros(0,bool)
        # warm active set from previous (shifted)
        if prevA[b] is None: wAl=np.zeros(n,bool); wAu=np.zeros(n,bool)
        else:
            pl,pu = prevA[b]
            def sh(v): o=v.copy(); o[:4*N]=np.concatenate([v[4:4*N], v[4*N-4:4*N]]); return o
            wAl, wAu = sh(pl), sh(pu)
        wp, itp, ok = pdas(q, wAl.copy(), wAu.copy())
        wc, itc, okc = pdas(q, np.zeros(n,bool), np.zeros(n,bool))
        feasC = (q["C"]@wp - q["c"]).min() if m else 0
        err = np.abs(wp-w).max()/max(1,np.abs(w).max())
        chg = (wAl!=Al).sum()+(wAu!=Au).sum()
        stats.append((st, Al.sum()+Au.sum(), Cact.sum(), chg, itp, ok, itc, okc, err, feasC, it))
        prevA[b]=(Al,Au)
    u0, diag, status = ffi.rti_step(kp, cfgv, N, M, K, x0, X, U, warm)
    x0 = X[:, 1, :].copy()
S=np.array(stats, dtype=float)
for st in range(STEPS):
    s=S[S[:,0]==st]
    print(f"step {st}: active {s[:,1].mean():5.1f} Cact {s[:,2].mean():4.2f} change {s[:,3].mean():5.2f} pdas_warm it {s[:,4].mean():4.2f} ok {s[:,5].mean():.2f} pdas_cold it {s[:,6].mean():4.2f} ok {s[:,7].mean():.2f} err max {s[:,8].max():.1e} minC {s[:,9].min():.1e} ipm {s[:,10].mean():.1f}")
