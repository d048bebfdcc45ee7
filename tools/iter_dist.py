"""Per-kite QP iteration counts along the bench workload (closed loop,
B = 4096, N = 20), saved to gpurun_out/iters.npz: input of the dispatch-order
(tail) analysis.  Tools only."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import openkite_amd as ok  # noqa: E402
from bench import synthetic_x0  # noqa: E402

B, STEPS = 4096, 14
g = ok.BatchNMPC(ok.load_properties(), ok.default_config(N=20), B)
x = synthetic_x0(B, 0, g)
its = []
for s in range(STEPS):
    r = g.step(x)
    its.append(g.qp_stats()[1].copy())
    x = r["traj"][:, 1, :].copy()
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(REPO, "gpurun_out", "iters.npz"), iters=np.array(its))
print("mean iterations per step", np.array(its).mean(axis=1))
g.close()
