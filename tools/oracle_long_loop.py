"""The bench's nominal closed loop (bench.py synthetic_x0, x0 <- traj[:, 1]
every step, N = 20, M = 2, K = 16) on the CPU oracle, per step: kites with
NaN (bit 1), restarts (64), rejected steps (32), state bound (8), QP at the
cap (2), and the worst |omega| / min airspeed.  CPU only (tools).
  python tools/oracle_long_loop.py [B] [steps] [threads] [N]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import ffi  # noqa: E402
import bench  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
S = int(sys.argv[2]) if len(sys.argv) > 2 else 60
T = int(sys.argv[3]) if len(sys.argv) > 3 else 8
N = int(sys.argv[4]) if len(sys.argv) > 4 else 20
kp = ffi.load_params()
cv = ffi.cfg_vector(ffi.node_config(N=N))


class _Ctx:
    def closest_point(self, pos):
        return np.array([ffi.closest_point(cv, p) for p in pos])


x = bench.synthetic_x0(B, 0, _Ctx())
X = np.zeros((B, N + 1, 15)); U = np.zeros((B, N, 4))
ever = np.zeros(B, dtype=np.int32)
for s in range(S):
    it = np.zeros(B, dtype=np.int32)
    _, d, st = ffi.rti_step(kp, cv, N, 2, 16, x, X, U, warm=int(s > 0), nthreads=T, iters=it)
    ever |= st
    x = X[:, 1, :].copy()
    fin = np.isfinite(x).all(axis=1)
    V = np.linalg.norm(x[fin, 0:3], axis=1)
    print(json.dumps(dict(step=s, nan=int(np.sum(st & 1 != 0)), restart=int(np.sum(st & 64 != 0)),
                          rejected=int(np.sum(st & 32 != 0)), bound=int(np.sum(st & 8 != 0)),
                          capped=int(np.sum(st & 2 != 0)), mean_it=round(float(it.mean()), 3),
                          max_w=round(float(np.abs(x[fin, 3:6]).max()), 3), min_V=round(float(V.min()), 3),
                          bad=[int(b) for b in np.where(st & (1 | 32 | 64))[0][:8]])), flush=True)
print("kites ever flagged:", {n: int(np.sum(ever & bit != 0)) for n, bit in
                               (("nan", 1), ("capped", 2), ("bound", 8), ("rejected", 32), ("restart", 64))})
