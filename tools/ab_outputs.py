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
    # bit patterns, so that NaN outputs (kites a failed step left non-finite)
    # compare equal when both builds produced the same NaN
    ne = {k: a[k].view(np.uint64) != b[k].view(np.uint64) for k in ("traj", "ctrl")}
    same = not any(m.any() for m in ne.values())
    fin = {k: np.isfinite(a[k]) & np.isfinite(b[k]) for k in ("traj", "ctrl")}
    d = max(float(np.abs(a[k] - b[k])[fin[k]].max(initial=0.0)) for k in ("traj", "ctrl"))
    first = min((int(np.argwhere(m)[0][0]) for m in ne.values() if m.any()), default=-1)
    print(f"bitwise {'EQUAL' if same else 'DIFFERENT'}; differing words {sum(int(m.sum()) for m in ne.values())}, "
          f"first differing step {first}; max finite |diff| {d:.3e}")
