"""Status statistics of the oracle's closed loop at N = 40 (BASELINE config 5's
horizon), 512 synthetic kites x 23 steps -- the same closed loop bench.py runs
(next measured state = the plan's node 1).  Tools only (CPU).

  python tools/oracle_n40_loop.py > profiles/<tag>_oracle_n40_closed_loop_status.txt
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ffi  # noqa: E402

kp = ffi.load_params()
N, B = 40, 512
cv = ffi.cfg_vector(ffi.node_config(N=N))
xs = ffi.synthetic_states(B)
x = np.zeros((B, 15)); x[:, :13] = xs
for b in range(B):
    x[b, 13] = ffi.closest_point(cv, xs[b, 6:9])
X = np.zeros((B, N + 1, 15)); U = np.zeros((B, N, 4))
qp_form = int(cv[77])
print(f"N = {N}, {B} kites x 23 steps, qp_form {qp_form} "
      f"({'multiple-shooting QP' if qp_form == 1 else 'condensed QP'})")
t = time.time()
for step in range(23):
    it = np.zeros(B, dtype=np.int32)
    u0, diag, st = ffi.rti_step(kp, cv, N, 2, 16, x, X, U, warm=int(step > 0), nthreads=8, iters=it)
    print(step, "nan", int(((st & 1) != 0).sum()), "restart", int(((st & 64) != 0).sum()),
          "rejected", int(((st & 32) != 0).sum()), "bound", int(((st & 8) != 0).sum()),
          "notconv", int(((st & 2) != 0).sum()), "mean_iters", round(float(it.mean()), 2))
    x = X[:, 1, :].copy()
print(f"{time.time() - t:.1f} s")
