"""Closed-loop study: is the synthetic fleet's loss of
speed a property of the OCP / the plant or of the RTI's single Gauss-Newton
iteration?  CPU oracle only (test infrastructure; no GPU).

The plant of every loop is the bench's: the next measured state is node 1 of
the committed plan (bench.py / openkite_amd/fleet.py), i.e. a perfect model.
Loops, same kites (bench.synthetic_x0 seeds) and steps:
  rti        the product: one RTI step per sampling instant (orc_rti_step)
  sqp        Gauss-Newton SQP iterated at every sampling instant until the full
             step is below 1e-4 (the reference's IPOPT tol, kiteNMPF.cpp:178-184)
             or 15 iterations, merit line search (orc_sqp_step)
  rti_T2     the RTI with twice the thrust box (ubu[0] 0.15 -> 0.30,
             nmpf_node.cpp:46-47)
  rti_lt     the RTI with a 4 m tether instead of umx_radian.yaml's 2.81 m
             (the orbit radius is 2.65 m, nmpf_node.cpp:31)
  rti_vref   the RTI with vref 2 instead of 4 (nmpf_node.cpp:68)
plus an open-loop run at full thrust with the surfaces at zero.

Per loop and step: min airspeed |v|, kites clamped at the min speed (status
bit 4: the prologue raised vx to 2.1), NaN (1), rejected (32), restart (64),
capped QPs (2), mean position error; then the first step at which half the
kites are at the clamp and the kite-steps lost.

    python tools/closed_loop_study.py [B] [steps] [threads] > profiles/r06_closed_loop_study.txt
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import ffi  # noqa: E402
import bench  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
S = int(sys.argv[2]) if len(sys.argv) > 2 else 100
T = int(sys.argv[3]) if len(sys.argv) > 3 else 8
N = 20
P_LT = 46                                  # tether length in the oracle's parameter vector (kite.h Lt)


class _Ctx:
    def __init__(self, cv):
        self.cv = cv

    def closest_point(self, pos):
        return np.array([ffi.closest_point(self.cv, p) for p in pos])


def run(name, kp, cfg, mode):
    cv = ffi.cfg_vector(cfg)
    x = bench.synthetic_x0(B, 0, _Ctx(cv))
    X = np.zeros((B, N + 1, 15)); U = np.zeros((B, N, 4))
    rows = []
    lost = np.zeros(B, dtype=bool)
    for s in range(S):
        warm = int(s > 0)
        if mode == "sqp":
            _, d, st, its, _ = ffi.sqp_step(kp, cv, N, 2, 16, x, X, U, warm=warm, maxit=15, tol=1e-4, nthreads=T)
            extra = dict(sqp_it=round(float(its.mean()), 2))
        else:
            _, d, st = ffi.rti_step(kp, cv, N, 2, 16, x, X, U, warm=warm, nthreads=T)
            extra = {}
        x = X[:, 1, :].copy()
        fin = np.isfinite(x).all(axis=1)
        V = np.linalg.norm(x[fin, 0:3], axis=1)
        lost |= (st & (1 | 32 | 64)) != 0
        r = dict(step=s, min_V=round(float(V.min()), 3) if V.size else None,
                 med_V=round(float(np.median(V)), 3) if V.size else None,
                 clamped=int(np.sum(st & 4 != 0)), nan=int(np.sum(st & 1 != 0)),
                 rejected=int(np.sum(st & 32 != 0)), restart=int(np.sum(st & 64 != 0)),
                 capped=int(np.sum(st & 2 != 0)), pos_err=round(float(np.nanmean(d[:, 0])), 4), **extra)
        rows.append(r)
    half = next((r["step"] for r in rows if r["clamped"] >= B // 2), None)
    first_fail = next((r["step"] for r in rows if r["nan"] + r["rejected"] + r["restart"] > 0), None)
    summ = dict(loop=name, kites=B, steps=S, first_step_half_clamped=half, first_step_with_failure=first_fail,
                kites_ever_failed=int(lost.sum()),
                kite_steps_failed=int(sum(r["nan"] + r["rejected"] + r["restart"] for r in rows)),
                min_V_at=[rows[i]["min_V"] for i in (0, 10, 20, 40, 60, S - 1) if i < S],
                med_V_at=[rows[i]["med_V"] for i in (0, 10, 20, 40, 60, S - 1) if i < S])
    return summ, rows


def open_loop(kp, cfg):
    """Full thrust, surfaces zero, 2 s, from the same launch states: the plant's
    own speed without a controller."""
    cv = ffi.cfg_vector(cfg)
    x = bench.synthetic_x0(B, 0, _Ctx(cv))
    u = np.array([cfg["ubu"][0], 0.0, 0.0, 0.0])
    out = []
    for t in range(40):
        x = np.array([ffi.rk4(kp, x[b], u, 0.025, 2) for b in range(B)])   # h = substep
        fin = np.isfinite(x).all(axis=1)
        V = np.linalg.norm(x[fin, 0:3], axis=1)
        out.append((round(0.05 * (t + 1), 2), round(float(V.min()), 3), round(float(np.median(V)), 3)))
    return out


def main():
    kp = ffi.load_params()
    base = ffi.node_config(N=N)
    print(__doc__.strip().splitlines()[0])
    print(f"B={B} kites, {S} steps of dt = {base['dt']} s, N = {N}, M = 2, K = 16, {T} threads")
    print("open loop, full thrust, surfaces 0: (t, min |v|, median |v|) =",
          [r for r in open_loop(kp, base)[::8]])
    loops = [("rti", kp, base, "rti"), ("sqp", kp, base, "sqp")]
    c = dict(base); c["ubu"] = list(base["ubu"]); c["ubu"][0] = 0.30
    loops.append(("rti_T2", kp, c, "rti"))
    kl = kp.copy(); kl[P_LT] = 4.0
    loops.append(("rti_lt", kl, base, "rti"))
    c = dict(base); c["vref"] = 2.0
    loops.append(("rti_vref", kp, c, "rti"))
    for name, k, cfg, mode in loops:
        summ, rows = run(name, k, cfg, mode)
        print(json.dumps(summ), flush=True)
        for r in rows[::5]:
            print("   ", json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
