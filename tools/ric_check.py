"""Quick GPU check of the multiple-shooting Riccati QP (qp_kernel 3) against
the oracle (qp_form 1): B kites, a cold step and warm steps from identical
inputs (the GPU restarts each step from the oracle's previous solution).

  python tools/ric_check.py [N] [B] [steps] [allbounds]

allbounds = 1: finite (wide) bounds on every kite state, so that every
interior node has 17 bounded variables (the NB = 13 register layout at N = 40).
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import openkite_amd as ok  # noqa: E402
from oracle import ffi  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 6
kp = ffi.load_params()
c = ffi.node_config(N=N)
c["qp_form"] = 1
allb = len(sys.argv) > 4 and sys.argv[4] == "1"
if allb:
    c["lbx"] = [v if np.isfinite(v) or i >= 13 else -50.0 for i, v in enumerate(c["lbx"])]
    c["ubx"] = [v if np.isfinite(v) or i >= 13 else 50.0 for i, v in enumerate(c["ubx"])]
cv = ffi.cfg_vector(c)
xs = ffi.synthetic_states(B)
x = np.zeros((B, 15)); x[:, :13] = xs
for b in range(B):
    x[b, 13] = ffi.closest_point(cv, xs[b, 6:9])
g = ok.BatchNMPC(ok.load_properties(), ok.default_config(N=N, qp_kernel=3), B)
if allb:
    g.set_bounds(np.array(c["lbx"]), np.array(c["ubx"]))
Xo = np.zeros((B, N + 1, 15)); Uo = np.zeros((B, N, 4))
try:
    for step in range(steps):
        if step > 0:
            g.set_solution(Xo, Uo)
        r = g.step(x)
        it = np.zeros(B, dtype=np.int32)
        u0, diag, st = ffi.rti_step(kp, cv, N, 2, 16, x, Xo, Uo, warm=int(step > 0), iters=it)
        kg, ig = g.qp_stats()
        d = np.abs(r["traj"] - Xo).reshape(B, -1).max(1) / np.maximum(1.0, np.abs(Xo).reshape(B, -1).max(1))
        cc = np.abs(r["ctrl"] - Uo).reshape(B, -1).max(1) / np.maximum(1.0, np.abs(Uo).reshape(B, -1).max(1))
        e = np.maximum(d, cc)
        print(f"step {step}: err median {np.median(e):.2e} max {e.max():.2e} | iters gpu {ig[:8]} oracle {it[:8]} "
              f"| kkt gpu {np.median(kg):.1e} oracle {np.median(diag[:, 5]):.1e} | status equal "
              f"{np.mean(r['status'] == st):.2f}", flush=True)
        if e.max() > 1e-6:
            b = int(np.argmax(e))
            print("  worst kite", b, "status", r["status"][b], st[b], "kkt", kg[b], diag[b, 5], "iters", ig[b], it[b])
            print("  u0 gpu", r["u0"][b], "oracle", u0[b])
        x = Xo[:, 1, :].copy()
finally:
    g.close()
