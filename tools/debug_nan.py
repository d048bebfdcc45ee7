"""Find instances that go non-finite in a B=4096 closed loop and replay them alone."""
import sys
sys.path.insert(0, ".")
import numpy as np
import openkite_amd as ok
from oracle import ffi
from tests.test_gpu_parity import x0_batch

B = 4096
cfg = ok.default_config()
g = ok.BatchNMPC(ok.load_properties(), cfg, B)
x = x0_batch(B)
hist = [x.copy()]
for step in range(3):
    r = g.step(x)
    kkt, it = g.qp_stats()
    bad = np.where(r["status"] & 1)[0]
    print("step", step, "nan instances", bad[:10], "kkt", kkt[bad[:10]] if len(bad) else None, "iters", it[bad[:10]] if len(bad) else None)
    if len(bad):
        b0 = bad[0]
        # replay: same warm state for that instance alone is not available -> replay from step 0 alone
        g1 = ok.BatchNMPC(ok.load_properties(), cfg, 1)
        xs = hist[0][b0:b0 + 1].copy()
        for s2 in range(step + 1):
            r1 = g1.step(xs)
            k1, i1 = g1.qp_stats()
            print("  alone step", s2, "status", r1["status"], "kkt", k1, "iters", i1)
            xs = r1["traj"][:, 1, :].copy()
        np.save("gpurun_out/nan_x0.npy", hist[0][b0])
        break
    x = r["traj"][:, 1, :].copy()
    hist.append(x.copy())
