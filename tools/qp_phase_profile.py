"""Phase profile of k_qp_tiled / k_qp_lds (s_memtime cycles per phase, mean per
instance).  Usage: qp_phase_profile.py [B] [N]

Runs the phase-instrumented build (make -C openkite_amd/csrc prof) on one
closed-loop bench-like workload.  Tools only: not part of the product path.
"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
os.environ.setdefault("KITE_NMPC_LIB", os.path.join(REPO, "openkite_amd", "lib", "libkite_nmpc_prof.so"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import openkite_amd as ok  # noqa: E402
from tests.test_gpu_parity import x0_batch  # noqa: E402

PHASES = ["init", "residual", "normal_matrix", "cholesky", "schur", "predictor", "corrector",
          "final_residual", "epilogue"]

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
NH = int(sys.argv[2]) if len(sys.argv) > 2 else 20
L = ok.lib()
L.kite_debug_qp_profile.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
buf = (ctypes.c_ulonglong * 16)()
g = ok.BatchNMPC(ok.load_properties(), ok.default_config(N=NH), B)
x = x0_batch(B)
for step in range(4):
    r = g.step(x)
    x = r["traj"][:, 1, :].copy()
L.kite_debug_cd_profile.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
cbuf = (ctypes.c_ulonglong * 8)()
L.kite_debug_qp_profile(buf)          # clear warm-up
L.kite_debug_cd_profile(cbuf)
r = g.step(x)
L.kite_debug_qp_profile(buf)
L.kite_debug_cd_profile(cbuf)
cv = np.array(cbuf[:8], dtype=np.float64)
print("k_condense (wave 0), cycles per instance:")
for i, nm in enumerate(["init", "node barrier", "W rows", "propagate", "fold", "output"]):
    print(f"  {nm:15s} {cv[i] / max(cv[7], 1):12.0f}")
v = np.array(buf[:16], dtype=np.float64)
ninst, its = v[10], v[9]
print(f"B={B} N={NH} instances={ninst:.0f} mean iterations={its / ninst:.2f}")
tot = v[:9].sum() / ninst
for i, p in enumerate(PHASES):
    c = v[i] / ninst
    per_it = c / (its / ninst) if i in (1, 2, 3, 4, 5, 6) else float("nan")
    print(f"{p:15s} {c:12.0f} cycles/instance  {100 * c / tot:5.1f}%  per-iteration {per_it:10.0f}")
print(f"{'total':15s} {tot:12.0f}")
if NH == 20:   # k_qp_tiled Cholesky sub-phases, cycles per instance
    for i, nm in enumerate(["stage panels", "panels", "trailing + next diagonal"]):
        print(f"  chol {nm:20s} {v[11 + i] / ninst:12.0f}")
if NH == 40:   # k_qp_lds sub-phases (wave 0 unless noted), cycles per instance
    for i, nm in enumerate(["load_h+symv", "diag tiles (wave 0)", "trailing (wave 1)", "panel", "msolve sweeps"]):
        print(f"  sub {nm:22s} {v[11 + i] / ninst:12.0f}")
g.close()
