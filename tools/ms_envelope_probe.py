"""Sensitivity envelope of the multiple-shooting QP (qp_form 1) on closed-loop
inputs: per kite and step, the oracle's MS QP solved on its own data and on the
data perturbed by a relative 1e-15 (two seeds); reports how far the frozen
solutions move (relative to max(1, |.|) of the physical trajectory update, the
quantity the GPU parity tests compare).  Tools only.
  python tools/ms_envelope_probe.py [B] [steps] [N] [z0]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ffi  # noqa: E402
from tests.test_gpu_parity import x0_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
Nh = int(sys.argv[3]) if len(sys.argv) > 3 else 40
z0 = float(sys.argv[4]) if len(sys.argv) > 4 else None
M, K = 2, 16
kp = ffi.load_params()
c = ffi.node_config(N=Nh)
cv = ffi.cfg_vector(c)
if z0 is not None:
    ffi.set_ms_z0(z0)
Sx = np.array(c["Sx"]) if "Sx" in c else None
x = x0_batch(B, offset=11000)
X = np.zeros((B, Nh + 1, 15)); U = np.zeros((B, Nh, 4))
errs, errs_same, its_diff, nfrozen, ncap = [], [], 0, 0, 0
worst = (0.0, None)
for step in range(steps):
    for b in range(B):
        st, Xp, Up, _ = ffi.prologue(kp, cv, Nh, M, x[b], X[b], U[b], warm=int(step > 0))
        v0, k0, i0 = ffi.msqp_solve(kp, cv, Nh, M, Xp, Up, K)
        for seed in (1, 2):
            v1, k1, i1 = ffi.msqp_solve_perturbed(kp, cv, Nh, M, Xp, Up, K, 1e-15, 1000 * b + 17 * step + seed)
            if k0 < 1e-10 and k1 < 1e-10:
                nfrozen += 1
                e = np.abs(v1 - v0).max() / max(1.0, np.abs(v0).max())
                errs.append(e)
                if i0 == i1:
                    errs_same.append(e)
                its_diff += int(i0 != i1)
                if e > worst[0]:
                    worst = (e, (step, b, seed, i0, i1, k0, k1))
            else:
                ncap += 1
    u0, diag, st = ffi.rti_step(kp, cv, Nh, M, K, x, X, U, warm=int(step > 0), nthreads=0)
    x = X[:, 1, :].copy()
e = np.array(errs)
print(f"N={Nh} z0={ffi.set_ms_z0(ffi.lib().orc_get_ms_z0())} B={B} steps={steps}: {nfrozen} perturbed solves "
      f"frozen on both sides ({ncap} not), iteration count changed in {its_diff}")
print(f"  relative change of v: median {np.median(e):.2e} p99 {np.quantile(e, 0.99):.2e} "
      f"p99.9 {np.quantile(e, 0.999):.2e} max {e.max():.2e}")
es = np.array(errs_same)
print(f"  same iteration count ({es.size}): median {np.median(es):.2e} p99.9 {np.quantile(es, 0.999):.2e} "
      f"max {es.max():.2e}")
print(f"  worst: {worst}")
