"""Per-phase device time vs batch size (HIP event ring over warm closed-loop
steps, torch-free): how the main QP kernel's time grows with the number of
kites per CU.  Tools only (GPU box).
  python tools/qp_scaling_probe.py [N] [steps] [B ...]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import openkite_amd as ok  # noqa: E402
from test_gpu_parity import x0_batch  # noqa: E402

Nh = int(sys.argv[1]) if len(sys.argv) > 1 else 20
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
Bs = [int(a) for a in sys.argv[3:]] or [1, 64, 256, 512, 1024, 2048, 4096]
xall = x0_batch(max(Bs))
for B in Bs:
    g = ok.BatchNMPC(ok.load_properties(), ok.default_config(N=Nh), B)
    x = xall[:B].copy()
    for _ in range(3):
        r = g.step(x)
        x = r["traj"][:, 1, :].copy()
    g.timing_start(steps)
    for _ in range(steps):
        r = g.step(x, want_traj=True)
        x = r["traj"][:, 1, :].copy()
    n, ks = g.timing_read()
    it = g.qp_iteration_sum() / float(B * steps)
    _, its = g.qp_stats()
    g.close()
    print(json.dumps(dict(B=B, N=Nh, steps=n, mean_iters=round(it, 3), max_iters_last=int(its.max()),
                          ms={k: round(v / max(1, n), 5) for k, v in ks.items()})), flush=True)
