"""Why the synthetic closed loop slows down (DESIGN 6,
"what the bench loop is"; tools/closed_loop_study.py,
profiles/r06_closed_loop_study.txt).  CPU oracle only.

The bench's plant is node 1 of the committed plan (a perfect model).  In that
loop every kite falls from ~5 m/s to the 2.1 m/s min-speed clamp
(nmpf_node.cpp:241-243) within ~22 steps.  These tests pin the cause:
  * the Gauss-Newton SQP iterated to the reference's IPOPT tolerance (1e-4,
    kiteNMPF.cpp:178-184) at every sampling instant decelerates exactly as the
    one-iteration RTI does -- the RTI semantics are not the cause;
  * the plant alone at the top of the thrust box (0.15, nmpf_node.cpp:46-47)
    with the surfaces at zero loses the same speed -- the launch state is
    faster than what the thrust box sustains.
"""
import numpy as np
import pytest

import bench
from oracle import ffi

N, M, K = 20, 2, 16
B, STEPS = 16, 26


class _Ctx:
    def __init__(self, cv):
        self.cv = cv

    def closest_point(self, pos):
        return np.array([ffi.closest_point(self.cv, p) for p in pos])


@pytest.fixture(scope="module")
def kp():
    return ffi.load_params()


def _loop(kp, cv, sqp):
    x = bench.synthetic_x0(B, 0, _Ctx(cv))
    X = np.zeros((B, N + 1, 15)); U = np.zeros((B, N, 4))
    minv, clamped, failed = [], [], 0
    for s in range(STEPS):
        if sqp:
            _, _, st, _, _ = ffi.sqp_step(kp, cv, N, M, K, x, X, U, warm=int(s > 0), maxit=15, tol=1e-4,
                                          nthreads=8)
        else:
            _, _, st = ffi.rti_step(kp, cv, N, M, K, x, X, U, warm=int(s > 0), nthreads=8)
        x = X[:, 1, :].copy()
        minv.append(float(np.linalg.norm(x[:, 0:3], axis=1).min()))
        clamped.append(int(np.sum((st & 4) != 0)))
        failed += int(np.sum((st & (1 | 32 | 64)) != 0))
    return np.array(minv), np.array(clamped), failed


def test_converged_sqp_decelerates_like_the_rti(kp):
    cv = ffi.cfg_vector(ffi.node_config(N=N))
    v_rti, c_rti, f_rti = _loop(kp, cv, sqp=False)
    v_sqp, c_sqp, f_sqp = _loop(kp, cv, sqp=True)
    assert f_rti == 0                                    # the headline's window is clean
    # both loops reach the clamp: every kite by the last step
    assert c_rti[-1] == B and c_sqp[-1] >= B - 1
    assert v_rti[0] > 4.0 and v_rti[20] < 2.3 and v_sqp[20] < 2.3
    # step by step the converged NLP's fleet is as slow as the RTI's
    assert np.max(np.abs(v_sqp - v_rti)) < 0.1, np.abs(v_sqp - v_rti)


def test_plant_alone_loses_the_launch_speed_at_full_thrust(kp):
    cv = ffi.cfg_vector(ffi.node_config(N=N))
    x = bench.synthetic_x0(B, 0, _Ctx(cv))
    u = np.array([0.15, 0.0, 0.0, 0.0])
    v0 = np.median(np.linalg.norm(x[:, 0:3], axis=1))
    for _ in range(33):                                  # 1.65 s at dt = 0.05
        x = np.array([ffi.rk4(kp, x[b], u, 0.025, 2) for b in range(B)])
    v1 = np.median(np.linalg.norm(x[:, 0:3], axis=1))
    assert v0 > 4.5 and v1 < 3.0, (v0, v1)
