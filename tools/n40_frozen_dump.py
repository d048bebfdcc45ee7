"""Dump for VERDICT r04 item 1: the sequence of
tests/test_gpu_parity.py::test_n40_qp_kernels_vs_oracle (16 kites, N = 40,
offset 7000, 4 warm steps from identical inputs, condensed QP kernels 1 and 2)
with, per step and kite, the GPU's own condensed QP data (kite_nmpc_get_qp),
the step inputs and both sides' plans, residuals and costs.  The analysis runs
on the CPU (tools/n40_frozen_analyse.py): the oracle's IPM is re-run on the
GPU's QP data, which separates the solver from the data.  Tools only (GPU box).
  python tools/n40_frozen_dump.py OUTDIR"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import openkite_amd as ok  # noqa: E402
from oracle import ffi  # noqa: E402
from test_gpu_parity import condensed_cfgv, x0_batch  # noqa: E402

out = sys.argv[1]
os.makedirs(out, exist_ok=True)
B, Nh, M, K = 16, 40, 2, 16
kp = ffi.load_params()
cv = condensed_cfgv(Nh)
for qk in (1, 2):
    cfg = ok.default_config(N=Nh)
    cfg.qp_kernel = qk
    g = ok.BatchNMPC(ok.load_properties(), cfg, B)
    x = x0_batch(B, offset=7000)
    Xo = np.zeros((B, Nh + 1, 15)); Uo = np.zeros((B, Nh, 4))
    d = {k: [] for k in ("x", "Xin", "Uin", "H", "h", "C", "cl", "cu", "traj_g", "ctrl_g", "diag_g", "kkt_g",
                         "it_g", "st_g", "traj_o", "ctrl_o", "diag_o", "st_o")}
    for step in range(4):
        Xin, Uin = Xo.copy(), Uo.copy()
        if step > 0:
            g.set_solution(Xo, Uo)
        r = g.step(x)
        kkt, it = g.qp_stats()
        qs = [g.get_qp(b) for b in range(B)]
        u0, diag, st = ffi.rti_step(kp, cv, Nh, M, K, x, Xo, Uo, warm=int(step > 0))
        for k, v in (("x", x), ("Xin", Xin), ("Uin", Uin), ("traj_g", r["traj"]), ("ctrl_g", r["ctrl"]),
                     ("diag_g", r["diag"]), ("kkt_g", kkt), ("it_g", it), ("st_g", r["status"]),
                     ("traj_o", Xo.copy()), ("ctrl_o", Uo.copy()), ("diag_o", diag), ("st_o", st)):
            d[k].append(np.array(v))
        for k in ("H", "h", "C", "cl", "cu"):
            d[k].append(np.stack([q[k] for q in qs]))
        e = np.array([max(np.abs(r["traj"][b] - Xo[b]).max() / max(1, np.abs(Xo[b]).max()),
                          np.abs(r["ctrl"][b] - Uo[b]).max() / max(1, np.abs(Uo[b]).max())) for b in range(B)])
        print(f"qp_kernel {qk} step {step}: plan errors {np.array2string(e, precision=1)}", flush=True)
        print(f"   kkt gpu {np.array2string(kkt, precision=1)}\n   kkt orc {np.array2string(diag[:, 5], precision=1)}",
              flush=True)
        x = Xo[:, 1, :].copy()
    g.close()
    np.savez_compressed(os.path.join(out, f"n40_frozen_qk{qk}.npz"), **{k: np.stack(v) for k, v in d.items()})
print("done", flush=True)
