"""Phase profile of k_qp_ric (s_memtime cycles per phase, mean per kite).
Usage: ric_phase_profile.py [B] [N]  (phase build: make -C openkite_amd/csrc prof)."""
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

PHASES = ["setup", "residual pass", "adjoint sweep", "sigma/rhs pass", "factor+pred backward",
          "pred forward", "affine ratio+mu_aff", "corrector rhs", "corr backward", "corr forward",
          "ratio+update", "final+commit"]
PER_IT = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10}
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
NH = int(sys.argv[2]) if len(sys.argv) > 2 else 20
L = ok.lib()
L.kite_debug_ric_profile.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
buf = (ctypes.c_ulonglong * 16)()
g = ok.BatchNMPC(ok.load_properties(), ok.default_config(N=NH), B)
x = x0_batch(B)
for step in range(4):
    r = g.step(x)
    x = r["traj"][:, 1, :].copy()
L.kite_debug_ric_subprofile.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
sub = (ctypes.c_ulonglong * 8)()
L.kite_debug_ric_profile(buf)          # clear warm-up
L.kite_debug_ric_subprofile(sub)
r = g.step(x)
L.kite_debug_ric_profile(buf)
L.kite_debug_ric_subprofile(sub)
v = np.array(buf[:16], dtype=np.float64)
nk, its = v[13], v[12]
print(f"B={B} N={NH} kites={nk:.0f} mean iterations={its / nk:.2f}")
tot = v[:12].sum() / nk
for i, p in enumerate(PHASES):
    c = v[i] / nk
    per_it = c / (its / nk) if i in PER_IT else float("nan")
    print(f"{p:22s} {c:12.0f} cycles/kite  {100 * c / tot:5.1f}%  per-iteration {per_it:10.0f}")
print(f"{'total':22s} {tot:12.0f}")
sv = np.array(sub[:8], dtype=np.float64) / nk / (its / nk) / NH
for i, nm in enumerate(["Z wait", "tail(k+1) + head(k)", "T, M MFMAs", "readlane/bcast/border", "chol4 + S", "transpose + rank-4", "carry"]):
    print(f"  factor stage: {nm:24s} {sv[i]:8.0f} cycles per stage")
g.close()
