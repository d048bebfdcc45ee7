"""Why fp32 sensitivities (config 4) cost IPM iterations.

Two contexts on the bench workload (4096 kites, N = 20): fp64 and fp32
sensitivities.  Run A (identical inputs): every step the fp32 context starts
from the fp64 context's solution (set_solution) and the same measured state,
so both condense the same linearisation point up to the fp32 rounding of
A_k, B_k -- differences in iteration counts are then caused by the perturbed
QP data alone.  Run B (free closed loops): each context follows its own
trajectory, as in the bench.  Prints mean iterations per step for both runs,
the condensed-H relative error of the fp32 QP against the fp64 QP at the same
point (64 kites), and the u0 difference.  Tools only.
  python tools/fp32_iter_probe.py [B] [STEPS]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import openkite_amd as ok  # noqa: E402
from bench import synthetic_x0  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 20
kp = ok.load_properties()
g64 = ok.BatchNMPC(kp, ok.default_config(N=20, qp_kernel=2), B)
g32 = ok.BatchNMPC(kp, ok.default_config(N=20, qp_kernel=2, sens_fp32=1), B)
x0 = synthetic_x0(B, 0, g64)

print("run A: identical inputs every step")
x = x0.copy()
itA64, itA32, herr, du = [], [], [], []
for s in range(STEPS):
    if s > 0:
        g32.set_solution(X64, U64)
    r64 = g64.step(x)
    r32 = g32.step(x)
    i64 = g64.qp_stats()[1].astype(float)
    i32 = g32.qp_stats()[1].astype(float)
    itA64.append(i64.mean()); itA32.append(i32.mean())
    if s in (1, STEPS // 2, STEPS - 1):
        e = []
        for b in range(0, B, max(1, B // 64)):
            H64 = g64.get_qp(b)["H"]; H32 = g32.get_qp(b)["H"]
            e.append(np.abs(H32 - H64).max() / np.abs(H64).max())
        herr.append((s, float(np.median(e)), float(np.max(e))))
    du.append(float(np.abs(r32["u0"] - r64["u0"]).max()))
    more = np.mean(i32 > i64); less = np.mean(i32 < i64)
    print(f"step {s:2d}: iterations fp64 {i64.mean():6.3f} fp32 {i32.mean():6.3f}  "
          f"kites fp32 more {more:.3f} fewer {less:.3f}  max |du0| {du[-1]:.2e}", flush=True)
    X64, U64 = r64["traj"].copy(), r64["ctrl"].copy()
    x = X64[:, 1, :].copy()
print(f"run A mean iterations (steps 1..): fp64 {np.mean(itA64[1:]):.3f} fp32 {np.mean(itA32[1:]):.3f}")
for s, med, mx in herr:
    print(f"  step {s}: condensed H relative error fp32 vs fp64 at the same point: median {med:.2e} max {mx:.2e}")

print("run B: free closed loops")
g64.reset(); g32.reset()
xa, xb = x0.copy(), x0.copy()
itB64, itB32 = [], []
for s in range(STEPS):
    ra = g64.step(xa); rb = g32.step(xb)
    itB64.append(g64.qp_stats()[1].mean()); itB32.append(g32.qp_stats()[1].mean())
    xa = ra["traj"][:, 1, :].copy(); xb = rb["traj"][:, 1, :].copy()
    print(f"step {s:2d}: iterations fp64 {itB64[-1]:6.3f} fp32 {itB32[-1]:6.3f}  "
          f"max |x_fp32 - x_fp64| {np.abs(xb - xa).max():.2e}", flush=True)
print(f"run B mean iterations (steps 1..): fp64 {np.mean(itB64[1:]):.3f} fp32 {np.mean(itB32[1:]):.3f}")
g64.close(); g32.close()
