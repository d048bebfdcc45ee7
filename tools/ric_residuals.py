"""Residual components of k_qp_ric's last convergence test per kite (phase
build, make -C openkite_amd/csrc prof), next to the oracle's iteration counts:
which part of max(rp, rg * dscale, mu) keeps a QP from freezing.
  python tools/ric_residuals.py [N] [B] [steps]"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
os.environ["KITE_NMPC_LIB"] = os.path.join(REPO, "openkite_amd", "lib", "libkite_nmpc_prof.so")
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import openkite_amd as ok  # noqa: E402
from oracle import ffi  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 40
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
L = ok.lib()
L.kite_debug_ric_residuals.argtypes = [ctypes.POINTER(ctypes.c_double)]
L.kite_debug_ric_trace.argtypes = [ctypes.POINTER(ctypes.c_double)]
buf = (ctypes.c_double * (4096 * 4))()
tbuf = (ctypes.c_double * (64 * 16 * 5))()
kp = ffi.load_params()
c = ffi.node_config(N=N)
c["qp_form"] = 1
cv = ffi.cfg_vector(c)
xs = ffi.synthetic_states(B)
x = np.zeros((B, 15)); x[:, :13] = xs
for b in range(B):
    x[b, 13] = ffi.closest_point(cv, xs[b, 6:9])
g = ok.BatchNMPC(ok.load_properties(), ok.default_config(N=N, qp_kernel=3), B)
Xo = np.zeros((B, N + 1, 15)); Uo = np.zeros((B, N, 4))
try:
    for step in range(steps):
        if step > 0:
            g.set_solution(Xo, Uo)
        r = g.step(x)
        assert L.kite_debug_ric_residuals(buf) == 0 and L.kite_debug_ric_trace(tbuf) == 0
        res = np.frombuffer(buf, dtype=np.float64).reshape(4096, 4)[:B]
        tr = np.frombuffer(tbuf, dtype=np.float64).reshape(64, 16, 5)
        Xp, Up = Xo.copy(), Uo.copy()
        it = np.zeros(B, dtype=np.int32)
        ffi.rti_step(kp, cv, N, 2, 16, x, Xo, Uo, warm=int(step > 0), iters=it)
        kg, ig = g.qp_stats()
        for b in range(B):
            e = np.abs(r["traj"][b] - Xo[b]).max() / max(1.0, np.abs(Xo[b]).max())
            flag = " <" if ig[b] != it[b] else ""
            print(f"step {step} kite {b:3d} it gpu {ig[b]:2d} orc {it[b]:2d} | rp {res[b, 0]:.1e} rg {res[b, 1]:.1e} "
                  f"mu {res[b, 2]:.1e} | err {e:.1e}{flag}")
            if flag and b < 64 and step == 0:
                _, Xl, Ul, _ = ffi.prologue(kp, cv, N, 2, x[b], Xp[b], Up[b], warm=int(step > 0))
                ffi.msqp_solve(kp, cv, N, 2, Xl, Ul, 16)
                ot = ffi.ms_trace()
                for i in range(max(ig[b], len(ot))):
                    gs = "  ".join(f"{v:9.2e}" for v in tr[b, i]) if i < min(16, ig[b]) else " " * 55
                    os_ = "  ".join(f"{v:9.2e}" for v in ot[i]) if i < len(ot) else ""
                    print(f"    it {i:2d} gpu r/mu/aa/sig/a {gs} | orc {os_}")
        x = Xo[:, 1, :].copy()
finally:
    g.close()
