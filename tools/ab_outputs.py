"""Closed-loop outputs of the library named by KITE_NMPC_LIB (B kites, N = 20,
S steps) saved to OUT.npz; with a second argument, compared bitwise with an
earlier run (tools only, A/B of library builds).
  python tools/ab_outputs.py OUT.npz [REF.npz] [B] [S] [N]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import openkite_amd as ok  # noqa: E402
from test_gpu_parity import x0_batch  # noqa: E402

out = sys.argv[1]
ref = sys.argv[2] if len(sys.argv) > 2 and sys.argv[2] != "-" else None
B = int(sys.argv[3]) if len(sys.argv) > 3 else 512
S = int(sys.argv[4]) if len(sys.argv) > 4 else 5
Nh = int(sys.argv[5]) if len(sys.argv) > 5 else 20
g = ok.BatchNMPC(ok.load_properties(), ok.default_config(N=Nh), B)
x = x0_batch(B)
trajs, ctrls = [], []
for _ in range(S):
    r = g.step(x)
    trajs.append(r["traj"]); ctrls.append(r["ctrl"])
    x = r["traj"][:, 1, :].copy()
g.close()
np.savez(out, traj=np.array(trajs), ctrl=np.array(ctrls))
if ref:
    a, b = np.load(ref), np.load(out)
    same = all(np.array_equal(a[k], b[k]) for k in ("traj", "ctrl"))
    d = max(float(np.abs(a[k] - b[k]).max()) for k in ("traj", "ctrl"))
    print(f"bitwise {'EQUAL' if same else 'DIFFERENT'}; max |diff| {d:.3e}")
