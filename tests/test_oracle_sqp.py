"""Oracle SQP continuation (orc_sqp_step, test infrastructure for the study in
DESIGN 9.3 / tools/sqp_study.py): Gauss-Newton SQP iterations at one sampling
instant with the kite state pinned to the processed measurement and the
theta relaxation box fixed at it (kiteNMPF.cpp:234-241 fixes the box at X0
for the whole NLP solve)."""
import numpy as np
import pytest

from oracle import ffi

M, K = 2, 16


@pytest.fixture(scope="module")
def kp():
    return ffi.load_params()


def _warm_plans(kp, cv, Nh, B, offset):
    from tests.test_gpu_parity import x0_batch
    x = x0_batch(B, offset=offset)
    X = np.zeros((B, Nh + 1, 15)); U = np.zeros((B, Nh, 4))
    for s in range(3):
        ffi.rti_step(kp, cv, Nh, M, K, x, X, U, warm=int(s > 0))
        x = X[:, 1, :].copy()
    return x, X, U


@pytest.mark.parametrize("Nh", [20, 40])
def test_sqp_first_iteration_is_the_rti_step(kp, Nh):
    """maxit = 1: bitwise the RTI step."""
    cv = ffi.cfg_vector(ffi.node_config(N=Nh))
    x, X, U = _warm_plans(kp, cv, Nh, 6, 9100 + Nh)
    X1, U1, X2, U2 = X.copy(), U.copy(), X.copy(), U.copy()
    _, d1, s1 = ffi.rti_step(kp, cv, Nh, M, K, x, X1, U1, warm=1)
    _, d2, s2, its, _ = ffi.sqp_step(kp, cv, Nh, M, K, x, X2, U2, warm=1, maxit=1, tol=0.0)
    np.testing.assert_array_equal(X1, X2)
    np.testing.assert_array_equal(U1, U2)
    np.testing.assert_array_equal(s1, s2)
    assert np.all(its == 1)


@pytest.mark.parametrize("ls", [0, 1])
def test_sqp_continuation_keeps_measurement_and_box(kp, ls):
    """After several iterations: the kite state at node 0 is the measurement
    bitwise, theta0 / thetadot0 stay inside the box around the measured
    values (not re-centred on each plan), the theta double integrator is exact,
    and the oracle's globals are restored (a following RTI step is unchanged)."""
    Nh, B = 20, 6
    c = ffi.node_config(N=Nh)
    cv = ffi.cfg_vector(c)
    x, X, U = _warm_plans(kp, cv, Nh, B, 9200)
    ffi.lib().orc_set_sqp(1e3, ls)
    try:
        Xs, Us = X.copy(), U.copy()
        ffi.sqp_step(kp, cv, Nh, M, K, x, Xs, Us, warm=1, maxit=6, tol=0.0)
    finally:
        ffi.lib().orc_set_sqp(1e3, 1)
    np.testing.assert_array_equal(Xs[:, 0, :13], x[:, :13])
    flex, dt = c["flex"], c["dt"]
    assert np.all(np.abs(Xs[:, 0, 13] - x[:, 13]) <= flex * (1 + 1e-12))
    assert np.all(np.abs(Xs[:, 0, 14] - x[:, 14]) <= flex * (1 + 1e-12))
    th, thd, uv = Xs[:, :-1, 13], Xs[:, :-1, 14], Us[:, :, 3]
    np.testing.assert_allclose(Xs[:, 1:, 13], th + dt * thd + 0.5 * dt * dt * uv, rtol=0, atol=1e-12)
    np.testing.assert_allclose(Xs[:, 1:, 14], thd + dt * uv, rtol=0, atol=1e-12)
    # globals restored: the plain RTI step is unaffected
    X1, U1, X2, U2 = X.copy(), U.copy(), X.copy(), U.copy()
    ffi.rti_step(kp, cv, Nh, M, K, x, X1, U1, warm=1)
    ffi.sqp_step(kp, cv, Nh, M, K, x, X2, U2, warm=1, maxit=1, tol=0.0)
    np.testing.assert_array_equal(X1, X2)


def test_sqp_converged_kite_is_a_fixed_point(kp):
    """A kite whose full step fell below 1e-9 has (numerically) stopped: a few
    more continuation iterations move its plan by less than 1e-7 (scaled)."""
    Nh, B = 20, 16
    c = ffi.node_config(N=Nh)
    cv = ffi.cfg_vector(c)
    x, X, U = _warm_plans(kp, cv, Nh, B, 9000)
    Xa, Ua = X.copy(), U.copy()
    _, _, st, its, step = ffi.sqp_step(kp, cv, Nh, M, K, x, Xa, Ua, warm=1, maxit=30, tol=1e-9)
    conv = step < 1e-9
    assert conv.sum() >= 1
    Xb, Ub = X.copy(), U.copy()
    ffi.sqp_step(kp, cv, Nh, M, K, x, Xb, Ub, warm=1, maxit=34, tol=0.0)
    Sx, Su = np.array(c["Sx"]), np.array(c["Su"])
    dx = np.abs((Xb - Xa) * Sx).reshape(B, -1).max(axis=1)
    du = np.abs((Ub - Ua) * Su).reshape(B, -1).max(axis=1)
    assert np.all(np.maximum(dx, du)[conv] < 1e-7), np.maximum(dx, du)[conv]
