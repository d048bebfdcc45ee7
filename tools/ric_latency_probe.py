"""Config 5 at its per-GPU shape (BASELINE configs[4]: 4096 kites / 8 GPUs =
512 per GPU, N = 40 + fused EKF): per timed step the QP kernel's time (HIP
events, kite_nmpc_timing_read) and the IPM iteration counts (mean, max) --
with one kite per SIMD the kernel lasts as long as its slowest kite.  Tools
only.   python tools/ric_latency_probe.py [B] [steps] [warmup]"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    import openkite_amd as ok
    from openkite_amd.fleet import FleetLoop, GpuStepper
    from bench import synthetic_x0

    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    W = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    N = 40
    dev = torch.device("cuda", 0)
    cfg = ok.default_config(N=N, M=2, qp_iters=16, device=0)
    ctx = ok.BatchNMPC(ok.load_properties(), cfg, B)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    x0 = synthetic_x0(B, 0, ctx)
    loop = FleetLoop(GpuStepper(ctx), torch.from_numpy(x0).to(dev), N, cfg.dt, ekf=True,
                     covariances=ok.ekf_default_covariances())
    for _ in range(W):
        loop.step()
    rows = []
    for s in range(S):
        ctx.timing_start(1, 1)
        loop.step()
        torch.cuda.synchronize(dev)
        nrec, ks = ctx.timing_read()
        it = ctx.qp_stats()[1]
        rows.append(dict(step=W + s, qp_main_ms=round(ks["qp_main"], 4), it_mean=round(float(it.mean()), 3),
                         it_max=int(it.max()), n_at_max=int(np.sum(it == it.max())),
                         ms_per_it_max=round(ks["qp_main"] / max(1, int(it.max())), 5)))
        print(json.dumps(rows[-1]), flush=True)
    q = np.array([r["qp_main_ms"] for r in rows])
    m = np.array([r["it_max"] for r in rows])
    print(json.dumps(dict(B=B, N=N, steps=S, qp_main_ms_mean=round(float(q.mean()), 4),
                          it_max_mean=round(float(m.mean()), 2),
                          us_per_iteration_of_slowest=round(float((q / m).mean()) * 1e3, 2))))
    ctx.close()


if __name__ == "__main__":
    main()
