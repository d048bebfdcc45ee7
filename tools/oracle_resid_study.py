"""Recursive residuals in the condensed IPM (the oracle cfg's qp_rec, k_qp_tiled's
rule): on the oracle's closed loop (N = 20,
qp_form 0, 512 synthetic kites x 23 steps), each step solved from the same
inputs with exact residuals (the product rule) and with recursive residuals
above a threshold; mean IPM iterations and the per-kite difference of the
committed step.  Tools only (CPU).   python tools/oracle_resid_study.py THR [THR ...]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ffi  # noqa: E402

kp = ffi.load_params()
N, B, STEPS = 20, 512, 23
base = dict(ffi.node_config(N=N), qp_form=0)
cv = ffi.cfg_vector(base)
xs = ffi.synthetic_states(B)
x = np.zeros((B, 15)); x[:, :13] = xs
for b in range(B):
    x[b, 13] = ffi.closest_point(cv, xs[b, 6:9])
thrs = [float(a) for a in sys.argv[1:]] or [1e-6]
X = np.zeros((B, N + 1, 15)); U = np.zeros((B, N, 4))
stats = {t: dict(it=0, d=[], diffit=0) for t in thrs}
it0_tot = 0
for step in range(STEPS):
    res = {}
    for t in [0.0] + thrs:
        ffi.lib().orc_reset_qp_recursive_counts()
        cvt = ffi.cfg_vector(dict(base, qp_rec=t))
        Xc, Uc = X.copy(), U.copy()
        it = np.zeros(B, dtype=np.int32)
        u0, diag, st = ffi.rti_step(kp, cvt, N, 2, 16, x, Xc, Uc, warm=int(step > 0), nthreads=8, iters=it)
        res[t] = (Xc, Uc, it, st)
        if t > 0:
            cnt = (ctypes.c_longlong * 2)()
            ffi.lib().orc_qp_recursive_counts(cnt)
            stats[t].setdefault("skips", 0); stats[t].setdefault("evals", 0)
            stats[t]["skips"] += cnt[0]; stats[t]["evals"] += cnt[1]
    Xe, Ue, ie, se = res[0.0]
    it0_tot += int(ie.sum())
    for t in thrs:
        Xr, Ur, ir, sr = res[t]
        d = np.maximum(np.abs(Xr - Xe).reshape(B, -1).max(1) / np.maximum(1, np.abs(Xe).reshape(B, -1).max(1)),
                       np.abs(Ur - Ue).reshape(B, -1).max(1) / np.maximum(1, np.abs(Ue).reshape(B, -1).max(1)))
        stats[t]["it"] += int(ir.sum()); stats[t]["d"].append(d); stats[t]["diffit"] += int(np.sum(ir != ie))
    X, U = Xe, Ue
    x = X[:, 1, :].copy()
print(f"exact residuals: mean iterations {it0_tot / (B * STEPS):.3f}")
for t in thrs:
    d = np.concatenate(stats[t]["d"])
    print(f"recursive above {t:g}: mean iterations {stats[t]['it'] / (B * STEPS):.3f}, "
          f"kite-steps with another count {stats[t]['diffit']} of {B * STEPS}, step difference: "
          f"median {np.median(d):.1e}, 99.9 % {np.quantile(d, 0.999):.1e}, max {d.max():.1e}, "
          f">1e-9: {int(np.sum(d > 1e-9))}; residual evaluations skipped {stats[t]['skips']} of "
          f"{stats[t]['skips'] + stats[t]['evals']}", flush=True)
