import sys
sys.path.insert(0, ".")
import numpy as np
import openkite_amd as ok
x0 = np.array([[4.181611752777922, 0.47684404179222967, 1.7609065814432234, 1.0681229501657965, -1.6928320420053362, -1.29099790517656, -0.4276135671632084, -2.6962544393702776, 0.6560016758768862, -0.02496333461727963, 0.16198953007576947, 0.4274073334474311, 0.8890777217915055, -1.5111472587692494, 0.0]])
for qk in (1, 2):
    cfg = ok.default_config(); cfg.qp_kernel = qk
    g = ok.BatchNMPC(ok.load_properties(), cfg, 1)
    x = x0.copy()
    for s in range(3):
        r = g.step(x); k, it = g.qp_stats()
        print("qp_kernel", qk, "step", s, "status", r["status"], "kkt", k, "iters", it)
        x = r["traj"][:, 1, :].copy()
