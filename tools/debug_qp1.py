"""Diagnostic: scalar (1) vs tiled (2) QP kernel, closed loop, several batch sizes."""
import sys
sys.path.insert(0, ".")
import numpy as np
import torch
import openkite_amd as ok
sys.path.insert(0, ".")
from tests.test_gpu_parity import x0_batch

for B in [16, 512, 4096]:
    x0 = x0_batch(B)
    for qk in [1, 2]:
        for dev_path in [False, True]:
            cfg = ok.default_config(); cfg.qp_kernel = qk
            g = ok.BatchNMPC(ok.load_properties(), cfg, B)
            x = x0.copy()
            out = []
            if dev_path:
                d_x0 = torch.from_numpy(x).cuda(); d_u0 = torch.zeros((B, 4), dtype=torch.float64, device="cuda")
                d_tr = torch.zeros((B, 21, 15), dtype=torch.float64, device="cuda")
                d_dg = torch.zeros((B, 6), dtype=torch.float64, device="cuda")
                d_st = torch.zeros((B,), dtype=torch.int32, device="cuda")
                g.set_stream(torch.cuda.current_stream().cuda_stream)
            for step in range(5):
                if dev_path:
                    g.step_device(d_x0.data_ptr(), d_u0.data_ptr(), d_tr.data_ptr(), 0, d_dg.data_ptr(), d_st.data_ptr())
                    d_x0.copy_(d_tr[:, 1, :]); torch.cuda.synchronize()
                    st = d_st.cpu().numpy(); u0 = d_u0.cpu().numpy()
                else:
                    r = g.step(x); st = r["status"]; u0 = r["u0"]; x = r["traj"][:, 1, :].copy()
                kkt, it = g.qp_stats()
                out.append(f"s{step}: nan={int(np.sum(st & 1))} it={it.mean():.2f} kkt_max={np.nanmax(kkt):.1e} u0[0]={u0[0,0]:.6f}")
            print(f"B={B} qk={qk} dev={dev_path}: " + " | ".join(out), flush=True)
            g.close()
