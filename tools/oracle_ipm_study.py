"""Step-to-boundary floor tau and start slack s0 of the condensed IPM (N = 20,
qp_form 0: the headline k_qp_tiled path) on the oracle's closed loop, 512
synthetic kites x 23 steps: mean IPM iterations and status counts.
Tools only (CPU).   python tools/oracle_ipm_study.py tau:s0 [tau:s0 ...]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ffi  # noqa: E402

kp = ffi.load_params()
N, B, STEPS = 20, 512, 23
cv = ffi.cfg_vector(ffi.node_config(N=N))
xs = ffi.synthetic_states(B, offset=int(os.environ.get("Z0_OFFSET", "0")))
x00 = np.zeros((B, 15)); x00[:, :13] = xs
for b in range(B):
    x00[b, 13] = ffi.closest_point(cv, xs[b, 6:9])
for arg in sys.argv[1:]:
    tau, s0 = (float(a) for a in arg.split(":"))
    ffi.set_ipm_study(tau, s0)
    x = x00.copy()
    X = np.zeros((B, N + 1, 15)); U = np.zeros((B, N, 4))
    tot = dict(nan=0, restart=0, rejected=0, bound=0, notconv=0, iters=0, capped=0)
    t = time.time()
    for step in range(STEPS):
        it = np.zeros(B, dtype=np.int32)
        u0, diag, st = ffi.rti_step(kp, cv, N, 2, 16, x, X, U, warm=int(step > 0), nthreads=8, iters=it)
        for k, bit in (("nan", 1), ("restart", 64), ("rejected", 32), ("bound", 8), ("notconv", 2)):
            tot[k] += int(((st & bit) != 0).sum())
        tot["iters"] += int(it.sum())
        tot["capped"] += int((it >= 16).sum())
        x = X[:, 1, :].copy()
    print(f"tau {tau:.4f} s0 {s0:6.3f}: mean_iters {tot['iters'] / (STEPS * B):.3f} capped {tot['capped']} "
          f"nan {tot['nan']} restart {tot['restart']} rejected {tot['rejected']} bound {tot['bound']} "
          f"notconv {tot['notconv']} ({time.time() - t:.1f} s)", flush=True)
ffi.set_ipm_study()
