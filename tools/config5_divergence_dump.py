"""Runs the config-5 sequence of tests/test_gpu_parity.py::_config5_vs_oracle
(B kites, N = 40 + fused EKF, GPU loop, oracle repeating each step from the GPU
loop's state) and saves the oracle inputs (x0, warm-start X, U) of every kite
whose step-safeguard decision or finiteness differs between GPU and oracle to
gpurun_out/<tag>/c5_diverged.npz.  Tools only (GPU box).
  python tools/config5_divergence_dump.py TAG [B] [steps] [offset]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402

import openkite_amd as ok  # noqa: E402
from openkite_amd.fleet import FleetLoop, GpuStepper  # noqa: E402
from oracle import ffi  # noqa: E402
from test_gpu_parity import x0_batch  # noqa: E402

tag = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
offset = int(sys.argv[4]) if len(sys.argv) > 4 else 12000
Nh, M, K = 40, 2, 16
kp = ffi.load_params()
cv = ffi.cfg_vector(ffi.node_config(N=Nh))
cfg = ok.default_config(N=Nh)
g = ok.BatchNMPC(ok.load_properties(), cfg, B)
W, V, P0 = ok.ekf_default_covariances()
g.set_stream(torch.cuda.current_stream().cuda_stream)
loop = FleetLoop(GpuStepper(g), torch.from_numpy(x0_batch(B, offset=offset)).cuda(), Nh, cfg.dt, ekf=True,
                 covariances=(W, V, P0))
dump = dict(x=[], X=[], U=[], step=[], kite=[], kkt_gpu=[], kkt_orc=[])
for step in range(steps):
    torch.cuda.synchronize()
    xe, P = loop.xe.cpu().numpy(), loop.P.cpu().numpy()
    u3, z, xin = loop.u0[:, :3].cpu().numpy(), loop.z.cpu().numpy(), loop.x0.cpu().numpy()
    Xo, Uo = g.get_solution() if step > 0 else (np.zeros((B, Nh + 1, 15)), np.zeros((B, Nh, 4)))
    loop.step()
    torch.cuda.synchronize()
    for b in range(B):
        for j in range(5):
            xe[b], P[b] = ffi.ekf_step(kp, xe[b], u3[b], cfg.dt / 5, P[b], z[b] if j == 4 else None, W, V)
    xin[:, :13] = xe
    Xi, Ui = Xo.copy(), Uo.copy()
    u0, diag, st = ffi.rti_step(kp, cv, Nh, M, K, xin, Xo, Uo, warm=int(step > 0), nthreads=0)
    stg = loop.status.cpu().numpy()
    kg, ko = loop.diag.cpu().numpy()[:, 5], diag[:, 5]
    bad = np.where(((stg & 32) != (st & 32)) | ~np.isfinite(kg) | ~np.isfinite(ko))[0]
    for b in bad:
        dump["x"].append(xin[b]); dump["X"].append(Xi[b]); dump["U"].append(Ui[b]); dump["step"].append(step)
        dump["kite"].append(b); dump["kkt_gpu"].append(kg[b]); dump["kkt_orc"].append(ko[b])
    print(step, "diverged", bad, kg[bad], ko[bad], flush=True)
g.close()
os.makedirs(f"gpurun_out/{tag}", exist_ok=True)
np.savez(f"gpurun_out/{tag}/c5_diverged.npz", **{k: np.array(v) for k, v in dump.items()})
