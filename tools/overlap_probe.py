"""Does splitting the batch over several streams overlap kernel tails?
(tools only)  python tools/overlap_probe.py [steps]

Times the closed-loop RTI step of 4096 kites as 1 x 4096, 2 x 2048 and
4 x 1024 contexts, each context on its own torch stream; prints RTI/s.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import openkite_amd as ok  # noqa: E402
from oracle import ffi  # noqa: E402

STEPS = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B, N = 4096, 20
cv = ffi.cfg_vector(ffi.node_config())
xs = ffi.synthetic_states(B)
x0 = np.zeros((B, 15)); x0[:, :13] = xs
for b in range(B):
    x0[b, 13] = ffi.closest_point(cv, xs[b, 6:9])
dev = torch.device("cuda:0")


def run(parts):
    n = B // parts
    lanes = []
    for p in range(parts):
        s = torch.cuda.Stream()
        ctx = ok.BatchNMPC(ok.load_properties(), ok.default_config(), n)
        ctx.set_stream(s.cuda_stream)
        x = torch.from_numpy(x0[p * n:(p + 1) * n].copy()).to(dev)
        lanes.append(dict(s=s, ctx=ctx, x=x, u0=torch.zeros((n, 4), dtype=torch.float64, device=dev),
                          traj=torch.zeros((n, N + 1, 15), dtype=torch.float64, device=dev),
                          diag=torch.zeros((n, 6), dtype=torch.float64, device=dev),
                          st=torch.zeros((n,), dtype=torch.int32, device=dev)))
    torch.cuda.synchronize()

    def step():
        for L in lanes:
            with torch.cuda.stream(L["s"]):
                L["ctx"].step_device(L["x"].data_ptr(), L["u0"].data_ptr(), L["traj"].data_ptr(), 0,
                                     L["diag"].data_ptr(), L["st"].data_ptr())
                L["x"].copy_(L["traj"][:, 1, :])

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(STEPS):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    for L in lanes:
        L["ctx"].close()
    return B * STEPS / dt, dt / STEPS * 1e3


for parts in (1, 2, 4, 1, 2, 4):
    v, ms = run(parts)
    print(f"{parts} x {B // parts}: {v:12.0f} RTI/s  {ms:.3f} ms/step", flush=True)
