"""Single-kite latency decomposition: for a batch-1
context at N = 20, a warm closed loop of `steps` steps, the wall time of
kite_nmpc_step (host arrays in and out, synchronous) and of
kite_nmpc_step_device + stream synchronisation, next to the device time of
every phase (config.timing = 1: HIP events of the last step), in episodes of
a reset + 25 warm steps as bench.py measures it.  Tools only.
  python tools/latency_probe.py [steps] [N] [batch]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import openkite_amd as ok  # noqa: E402
from test_gpu_parity import x0_batch  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
Nh = int(sys.argv[2]) if len(sys.argv) > 2 else 20
Bt = int(sys.argv[3]) if len(sys.argv) > 3 else 1
# phases: a timing context (cfg.timing = 1 records the events, so it runs the
# plain launch sequence); the wall time: a default context (captured step)
gt = ok.BatchNMPC(ok.load_properties(), ok.default_config(N=Nh, timing=1), Bt)
g = ok.BatchNMPC(ok.load_properties(), ok.default_config(N=Nh), Bt)
xs0 = x0_batch(max(Bt, 40))
EP = 25        # episodes of one cold step (reset, untimed) + EP warm steps, as bench.py: the
               # synthetic plant leaves the feasible region after ~45-150 steps


def episodes(n_timed, run):
    """run(first_state) -> list of per-step wall times of EP warm steps."""
    out, e = [], 0
    while len(out) < n_timed + 20:
        xe = np.roll(xs0, -e * Bt, axis=0)[:Bt]
        out += run(xe.copy())
        e += 1
    return out[20:20 + n_timed]


wall, wall_t, ph = [], [], []


def host_episode(x):
    g.reset(); gt.reset()
    r = g.step(x); rt = gt.step(x)
    x, xt = r["traj"][:, 1, :].copy(), rt["traj"][:, 1, :].copy()
    ts = []
    for _ in range(EP):
        t0 = time.perf_counter()
        r = g.step(x)
        t1 = time.perf_counter()
        rt = gt.step(xt)
        t2 = time.perf_counter()
        x, xt = r["traj"][:, 1, :].copy(), rt["traj"][:, 1, :].copy()
        ts.append(t1 - t0)
        wall_t.append(t2 - t1)
        ph.append(gt.kernel_times())
        if not (np.isfinite(x).all() and np.isfinite(xt).all()):
            break
    return ts


wall = episodes(steps, host_episode)
gt.close()
out = dict(batch=Bt, N=Nh, steps=steps, episode=EP, host_step_median_ms=float(np.median(wall) * 1e3),
           host_step_p90_ms=float(np.percentile(wall, 90) * 1e3),
           host_step_timed_plain_median_ms=float(np.median(wall_t) * 1e3),
           phases_median_ms={k: float(np.median([p[k] for p in ph])) for k in ph[0]})
# device entry point on torch's stream, synchronised per step (inputs in HBM)
g.set_stream(torch.cuda.current_stream().cuda_stream)
d_u = torch.zeros((Bt, 4), dtype=torch.float64, device="cuda")
d_t = torch.zeros((Bt, Nh + 1, 15), dtype=torch.float64, device="cuda")
d_d = torch.zeros((Bt, 6), dtype=torch.float64, device="cuda")
d_s = torch.zeros((Bt,), dtype=torch.int32, device="cuda")


def device_episode(x):
    g.reset()
    d_x = torch.from_numpy(x).cuda()
    g.step_device(d_x.data_ptr(), d_u.data_ptr(), d_t.data_ptr(), 0, d_d.data_ptr(), d_s.data_ptr())
    torch.cuda.synchronize()
    d_x.copy_(d_t[:, 1, :])
    ts = []
    for _ in range(EP):
        t0 = time.perf_counter()
        g.step_device(d_x.data_ptr(), d_u.data_ptr(), d_t.data_ptr(), 0, d_d.data_ptr(), d_s.data_ptr())
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
        d_x.copy_(d_t[:, 1, :])
    return ts


wd = episodes(steps, device_episode)
out["device_step_median_ms"] = float(np.median(wd) * 1e3)
out["device_step_p90_ms"] = float(np.percentile(wd, 90) * 1e3)
g.close()
print(json.dumps(out), flush=True)
