"""Timeline of the two-wave k_qp_ric (s_memtime at the hand-over points of
both waves; the first 4 dispatch slots, which the LPT order gives to the kites
with the most IPM iterations).  Needs the phase build without the factor
sub-markers:  make -C openkite_amd/csrc prof2.
Usage: ric_timeline.py [B] [N]   (B <= 2 x CUs so that the two-wave kernel runs)."""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
os.environ.setdefault("KITE_NMPC_LIB", os.path.join(REPO, "openkite_amd", "lib", "libkite_nmpc_prof2.so"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import openkite_amd as ok  # noqa: E402
from tests.test_gpu_parity import x0_batch  # noqa: E402

EV = 18
NAMES = {
    8: "M Sigma + test published (1)",
    0: "S has Sigma (1)",
    1: "S factor done",
    9: "M pred vector backward done",
    2: "S past (4)",
    10: "M past (4)",
    3: "S pred forward done",
    11: "M affine ratio + mu_aff done",
    12: "M corrector rhs done",
    4: "S past (5)",
    13: "M past (5)",
    5: "S corr backward done",
    14: "M feed-forward done",
    6: "S past (5b)",
    15: "M past (5b)",
    7: "S corr forward done",
    16: "M corrector ratio done",
    17: "M update done (iteration end)",
}
ORDER = [8, 0, 1, 9, 2, 10, 3, 11, 12, 4, 13, 5, 14, 6, 15, 7, 16, 17]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    NH = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    L = ok.lib()
    L.kite_debug_ric_timeline.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    buf = (ctypes.c_ulonglong * (4 * 16 * EV))()
    g = ok.BatchNMPC(ok.load_properties(), ok.default_config(N=NH), B)
    x = x0_batch(B)
    for _ in range(4):
        r = g.step(x)
        x = r["traj"][:, 1, :].copy()
    L.kite_debug_ric_timeline(buf)                  # clear
    g.step(x)
    L.kite_debug_ric_timeline(buf)
    t = np.array(buf[:], dtype=np.float64).reshape(4, 16, EV)
    rows = []
    for s in range(4):
        n = int(np.sum(t[s, :, 17] > 0))
        # iterations 1 .. n-1 (start = the previous iteration's end)
        for it in range(1, n):
            t0 = t[s, it - 1, 17]
            if np.all(t[s, it, :] > 0):
                rows.append(t[s, it, :] - t0)
        print(f"slot {s}: {n} full iterations")
    R = np.array(rows)
    print(f"B={B} N={NH}: {len(R)} iterations (slots 0-3, iteration >= 1); cycles from the iteration start, mean (min, max)")
    prev = 0.0
    for e in ORDER:
        m = R[:, e].mean()
        print(f"  {NAMES[e]:34s} {m:9.0f}  (+{m - prev:7.0f})   [{R[:, e].min():8.0f}, {R[:, e].max():8.0f}]")
        prev = m
    g.close()


if __name__ == "__main__":
    main()
