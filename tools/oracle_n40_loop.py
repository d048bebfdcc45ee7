"""Status statistics of the oracle's closed loop at N = 40 (BASELINE config 5's
horizon), 512 synthetic kites x 23 steps -- the same closed loop bench.py runs
(next measured state = the plan's node 1).  Tools only (CPU).

  python tools/oracle_n40_loop.py [z0] > profiles/<tag>_oracle_n40_closed_loop_status.txt
(z0: start multiplier of the multiple-shooting IPM, default the oracle's MS_Z0)
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ffi  # noqa: E402

kp = ffi.load_params()
if len(sys.argv) > 1:
    ffi.set_ms_z0(float(sys.argv[1]))
N, B = 40, 512
cv = ffi.cfg_vector(ffi.node_config(N=N))
xs = ffi.synthetic_states(B)
x = np.zeros((B, 15)); x[:, :13] = xs
for b in range(B):
    x[b, 13] = ffi.closest_point(cv, xs[b, 6:9])
X = np.zeros((B, N + 1, 15)); U = np.zeros((B, N, 4))
qp_form = int(cv[77])
z0 = ffi.set_ms_z0(ffi.lib().orc_get_ms_z0())
tot = dict(nan=0, restart=0, rejected=0, bound=0, notconv=0, iters=0)
print(f"N = {N}, {B} kites x 23 steps, qp_form {qp_form}, z0 {z0} "
      f"({'multiple-shooting QP' if qp_form == 1 else 'condensed QP'})")
t = time.time()
for step in range(23):
    it = np.zeros(B, dtype=np.int32)
    u0, diag, st = ffi.rti_step(kp, cv, N, 2, 16, x, X, U, warm=int(step > 0), nthreads=8, iters=it)
    print(step, "nan", int(((st & 1) != 0).sum()), "restart", int(((st & 64) != 0).sum()),
          "rejected", int(((st & 32) != 0).sum()), "bound", int(((st & 8) != 0).sum()),
          "notconv", int(((st & 2) != 0).sum()), "mean_iters", round(float(it.mean()), 2))
    for k, bit in (("nan", 1), ("restart", 64), ("rejected", 32), ("bound", 8), ("notconv", 2)):
        tot[k] += int(((st & bit) != 0).sum())
    tot["iters"] += int(it.sum())
    x = X[:, 1, :].copy()
print(f"total over {23 * B} kite-steps: nan {tot['nan']} restart {tot['restart']} rejected {tot['rejected']} "
      f"bound {tot['bound']} notconv {tot['notconv']} mean_iters {tot['iters'] / (23 * B):.3f}")
print(f"{time.time() - t:.1f} s")
