"""Oracle study: Gauss-Newton SQP iterated to convergence at one sampling
instant (oracle orc_sqp_step; the reference iterates IPOPT with an exact
Hessian to tol 1e-4 per control step, kiteNMPF.cpp:178-184, :286).

64 kites after 5 closed-loop RTI steps (node configuration), then up to
`maxit` SQP iterations at the 6th sampling instant with the theta box fixed at
the processed measurement (kiteNMPF.cpp:234-241).  Reports the fraction of
kites whose last full step (scaled inf-norm over the plan) is below 1e-4 /
1e-6, for full steps and for a backtracking line search on the merit
cost + nu * L1(defects, state-bound violations), LM damping off in the
continuation iterations.  CPU only (test infrastructure).

    python tools/sqp_study.py > profiles/r04_oracle_sqp_study.txt
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import ffi  # noqa: E402
from tests.test_gpu_parity import x0_batch  # noqa: E402

B = 64
kp = ffi.load_params()
print(__doc__.strip().splitlines()[0])
print(f"B={B}, warm plans after 5 RTI steps, tol 1e-6 stop, nu = 1e3")
for ls in (0, 1):
    ffi.lib().orc_set_sqp(1e3, ls)
    for Nh, form in ((20, 0), (20, 1), (40, 1)):
        c = ffi.node_config(N=Nh)
        c["qp_form"] = form
        cv = ffi.cfg_vector(c)
        x = x0_batch(B, offset=9000)
        X = np.zeros((B, Nh + 1, 15)); U = np.zeros((B, Nh, 4))
        for s in range(5):
            ffi.rti_step(kp, cv, Nh, 2, 16, x, X, U, warm=int(s > 0), nthreads=8)
            x = X[:, 1, :].copy()
        c["lm"] = 0.0
        cv = ffi.cfg_vector(c)
        for maxit in (10, 40):
            X2 = X.copy(); U2 = U.copy()
            _, diag, st, its, step = ffi.sqp_step(kp, cv, Nh, 2, 16, x, X2, U2, warm=1, maxit=maxit, tol=1e-6,
                                                  nthreads=8)
            fin = np.isfinite(step)
            print(f"{'line search' if ls else 'full steps '} N={Nh} qp_form={form} maxit={maxit:2d}: "
                  f"step<1e-4 {np.mean(step < 1e-4):.3f}  step<1e-6 {np.mean(step < 1e-6):.3f}  "
                  f"median step {np.median(step[fin]):.2e}  NaN {int(np.sum(st & 1))}  "
                  f"rejected {int(np.sum((st & 32) != 0))}  mean iterations {its.mean():.2f}", flush=True)
ffi.lib().orc_set_sqp(1e3, 1)
