"""CPU tests of the parity oracle (oracle/kite_oracle.cpp).

The oracle is pinned by the golden fixtures (50-digit sympy/mpmath
restatement of kite.cpp / kitemath.cpp / chebyshev.hpp, tests/golden/) and by
textbook Chebyshev values.  The reference's own tests hold no expected values
(every case ends in BOOST_CHECK(true)); their inputs are reused.
"""
import math

import numpy as np
import pytest

from oracle import ffi

RHS_TOL = 1e-13     # relative, f
JAC_TOL = 1e-12     # relative, df/d[x,u]
RK4_TOL = 1e-12     # relative, x+
SENS_TOL = 1e-10    # relative, S = dx+/d[x,u]


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.abs(a - b).max() / max(1.0, np.abs(b).max())


def test_rhs_matches_golden(kp, golden):
    for c in golden["rhs"]:
        assert rel(ffi.rhs(kp, c["x"], c["u"]), c["f"]) < RHS_TOL, c["source"]


def test_rti_cost_matches_golden(golden):
    """The RTI objective (sum of the squared GN residuals of every node plus
    the control term, oracle traj_cost) against the reference's Lagrange and
    Mayer terms restated at 50 digits with the node's weights, scaling,
    reference speed and path (kiteNMPF.cpp:117-141, nmpf_node.cpp:30-68)."""
    cv = ffi.cfg_vector(ffi.node_config(N=20))
    for c in golden["rti_cost"]["cases"]:
        J = ffi.traj_cost(cv, 20, np.array(c["X"]), np.array(c["U"]))
        assert abs(J - c["J"]) <= 1e-13 * c["J"], (J, c["J"])


@pytest.mark.parametrize("method", ["ad", "cs"])
def test_jacobian_matches_golden(kp, golden, method):
    for c in golden["rhs"]:
        J = ffi.rhs_jac(kp, c["x"], c["u"], method)
        assert rel(J, c["J"]) < JAC_TOL, (method, c["source"])


def test_rk4_and_sensitivities_match_golden(kp, golden):
    for c in golden["rk4"]:
        xo, A, B = ffi.rk4_sens(kp, c["x"], c["u"], c["tf"] / c["M"], c["M"])
        assert rel(xo, c["xnext"]) < RK4_TOL, c["source"]
        assert rel(A, c["A"]) < SENS_TOL, c["source"]
        assert rel(B, c["B"]) < SENS_TOL, c["source"]


def test_reference_rk4_call(kp, golden):
    """ODESolver::rk4_solve one step of 7 s (kite_model_test.cpp:58-75): diverges
    to ~1e62, which both the oracle and the 50-digit restatement reproduce."""
    c = golden["rk4_reference_call"]
    xo = ffi.rk4(kp, c["x"], c["u"], c["tf"], 1)
    np.testing.assert_allclose(xo, c["xnext"], rtol=1e-12)


def test_ad_matches_complex_step_through_rk4(kp):
    x = np.r_[ffi.BASE_STATE, 1.1, -0.2]
    for M in (1, 2, 4):
        _, A, B = ffi.rk4_sens(kp, x, [0.12, 0.05, -0.03, 1.5], 0.05 / M, M)
        Ac, Bc = ffi.rk4_sens_cs(kp, x, [0.12, 0.05, -0.03, 1.5], 0.05 / M, M)
        assert rel(A, Ac) < 1e-13 and rel(B, Bc) < 1e-13


def test_theta_double_integrator_is_exact(kp):
    """theta' = thetadot, thetadot' = Uv (kiteNMPF.cpp:62-73): RK4 is exact."""
    x = np.r_[ffi.BASE_STATE, 0.7, -1.3]
    u = [0.12, 0.0, 0.0, 2.5]
    T = 0.05
    xo, A, B = ffi.rk4_sens(kp, x, u, T / 2, 2)
    assert xo[13] == pytest.approx(0.7 - 1.3 * T + 0.5 * T * T * 2.5, abs=1e-15)
    assert xo[14] == pytest.approx(-1.3 + T * 2.5, abs=1e-15)
    assert A[13, 14] == pytest.approx(T) and B[13, 3] == pytest.approx(0.5 * T * T) and B[14, 3] == pytest.approx(T)


def test_chebyshev_golden_and_textbook(golden):
    ch = golden["chebyshev"]
    for n, D in ch["D"].items():
        np.testing.assert_allclose(ffi.cheb_D(int(n)), D, atol=1e-12)
    for n, w in ch["weights"].items():
        np.testing.assert_allclose(ffi.cheb_weights(int(n)), w, atol=1e-14)
        assert sum(w) == pytest.approx(2.0)
    for n, x in ch["points"].items():
        np.testing.assert_allclose(ffi.cheb_points(int(n)), x, atol=1e-15)
    np.testing.assert_allclose(ffi.cheb_compD(5, 2), ch["compD"]["5x2"], atol=1e-12)
    np.testing.assert_allclose(ffi.cheb_compD(2, 3), ch["compD"]["2x3"], atol=1e-12)
    tb = ch["textbook"]
    np.testing.assert_allclose(ffi.cheb_D(2), tb["D2"], atol=1e-14)
    np.testing.assert_allclose(ffi.cheb_D(5)[0], tb["D5_row0"], atol=1e-6)
    np.testing.assert_allclose(ffi.cheb_weights(5), tb["w5"], atol=1e-6)
    np.testing.assert_allclose(ffi.cheb_weights(2), tb["w2"], atol=1e-14)
    e = ch["expansion"]
    assert ffi.cheb_expansion(e["coef"], e["x"]) == pytest.approx(e["value"])
    assert math.isinf(ffi.lib().orc_cheb_expansion(None, 0, 0.5))


def test_path_matches_golden(golden):
    pc = golden["path"]
    cfg = ffi.node_config()
    cv = ffi.cfg_vector(cfg)
    assert cfg["path_R"] == pc["radius"]
    for c in pc["cases"]:
        P, dP = ffi.path(cv, c["theta"])
        np.testing.assert_allclose(P, c["P"], atol=1e-14)
        np.testing.assert_allclose(dP, c["dP"], atol=1e-14)


def test_closest_point_behaviour(cfgv):
    """kiteNMPF.cpp:358-391: <= 11 gradient steps of 0.25 on 0.5*||P - r||."""
    P, _ = ffi.path(cfgv, 1.0)
    pos = P * 1.05
    th = ffi.closest_point(cfgv, pos, 0.3)
    d_before = np.linalg.norm(ffi.path(cfgv, 0.3)[0] - pos)
    d_after = np.linalg.norm(ffi.path(cfgv, th)[0] - pos)
    assert d_after < d_before and abs(th - 1.0) < 0.3
    # a guess with (near) zero gradient triggers the restart from pi/2 + 0.1
    P0, _ = ffi.path(cfgv, 0.0)
    th2 = ffi.closest_point(cfgv, P0 * 1.05, 0.0)
    assert th2 != 0.0 and abs(th2) < math.pi / 2 + 0.1


def _cold_instances(kp, cv, B):
    xs = ffi.synthetic_states(B)
    x0 = np.zeros((B, 15))
    x0[:, :13] = xs
    for b in range(B):
        x0[b, 13] = ffi.closest_point(cv, xs[b, 6:9])
    return x0


def test_prologue_cold_and_shift(kp, cfgv):
    N, M = 20, 2
    x0 = _cold_instances(kp, cfgv, 1)[0]
    st, X, U, xo = ffi.prologue(kp, cfgv, N, M, x0, np.zeros((N + 1, 15)), np.zeros((N, 4)), warm=0)
    assert st == 0
    np.testing.assert_array_equal(X[0], x0)
    np.testing.assert_allclose(U, np.tile([0.125, 0.0, 0.0, 0.0], (N, 1)))
    for k in range(N):   # cold start is a forward simulation: no defects
        np.testing.assert_allclose(X[k + 1], ffi.rk4(kp, X[k], U[k], 0.025, 2), atol=1e-14)
    # warm + shift: X_k <- X_{k+1}, last node duplicated, theta re-simulated
    U2 = U.copy(); U2[:, 3] = np.linspace(-1, 1, N)
    x1 = X[1].copy(); x1[13] = 7.0        # > 2 pi -> wrapped
    st, Xs, Us, xo = ffi.prologue(kp, cfgv, N, M, x1, X, U2, warm=1)
    assert st & 16
    assert xo[13] == pytest.approx(7.0 - 2 * math.pi)
    np.testing.assert_array_equal(Xs[5, :13], X[6, :13])
    np.testing.assert_array_equal(Us[:-1], U2[1:])


def test_min_speed_clamp(kp, cfgv):
    x0 = _cold_instances(kp, cfgv, 1)[0]
    x0[0] = 1.0
    st, X, U, xo = ffi.prologue(kp, cfgv, 20, 2, x0, np.zeros((21, 15)), np.zeros((20, 4)), warm=0)
    assert st & 4 and xo[0] == 2.1


def test_qp_kkt_and_bounds(kp, cfgv):
    N, M = 20, 2
    x0 = _cold_instances(kp, cfgv, 2)
    for b in range(2):
        st, X, U, _ = ffi.prologue(kp, cfgv, N, M, x0[b], np.zeros((N + 1, 15)), np.zeros((N, 4)), warm=0)
        q = ffi.build_qp(kp, cfgv, N, M, X, U)
        H = q["H"]
        assert np.allclose(H, H.T, atol=1e-9 * np.abs(H).max())
        assert np.linalg.eigvalsh(H).min() > 0
        w, kkt = ffi.qp_solve(H, q["h"], q["lb"], q["ub"], q["C"], q["c"], 30)
        assert kkt < 1e-9
        assert np.all(w >= q["lb"] - 1e-9) and np.all(w <= q["ub"] + 1e-9)
        assert np.all(q["C"] @ w >= q["c"] - 1e-8)


def test_rti_closed_loop_is_stable(kp, cfgv):
    N, M, K, B = 20, 2, 16, 8
    x = _cold_instances(kp, cfgv, B)
    X = np.zeros((B, N + 1, 15)); U = np.zeros((B, N, 4))
    for step in range(12):
        u0, diag, st = ffi.rti_step(kp, cfgv, N, M, K, x, X, U, warm=int(step > 0))
        assert np.all(np.isfinite(diag)) and not np.any(st & 1)
        assert np.all(diag[:, 5] < 1e-8)           # QP converged within K
        assert np.all(u0 >= np.array([0.1, -0.1222, -0.1222, -5]) - 1e-6)
        x = X[:, 1, :].copy()                       # nominal closed loop
    # the RTI converged iterate is a fixed point of the step (no change when
    # re-solved at the same initial state without shift)


def test_rti_is_deterministic_and_batch_invariant(kp, cfgv):
    N, M, K = 20, 2, 16
    x = _cold_instances(kp, cfgv, 6)
    X1 = np.zeros((6, N + 1, 15)); U1 = np.zeros((6, N, 4))
    u1, d1, s1 = ffi.rti_step(kp, cfgv, N, M, K, x, X1, U1, warm=0, nthreads=4)
    X2 = np.zeros((2, N + 1, 15)); U2 = np.zeros((2, N, 4))
    u2, d2, s2 = ffi.rti_step(kp, cfgv, N, M, K, x[3:5].copy(), X2, U2, warm=0, nthreads=1)
    np.testing.assert_array_equal(u1[3:5], u2)
    np.testing.assert_array_equal(X1[3:5], X2)


def test_qp_sensitivity_envelope(kp, cfgv):
    """Intrinsic sensitivity of the condensed QP (sets COND_ENVELOPE of
    test_gpu_parity.py): symmetric relative perturbations of H of 1e-15 --
    rounding-level differences between two fp64 implementations -- move the
    oracle's own frozen QP solution by up to ~2e-6 (cond(H) ~ 1e11): 64
    closed-loop kites x 6 steps here, median ~1e-10; 1024 solves measured max
    2.0e-6 at the former z0 = 10 and 6.9e-7 at z0 = 20."""
    from tests.test_gpu_parity import COND_ENVELOPE, x0_batch
    N, M, K, B = 20, 2, 16, 64
    x = x0_batch(B, offset=2000)
    X = np.zeros((B, N + 1, 15)); U = np.zeros((B, N, 4))
    errs = []
    for step in range(6):
        for b in range(B):
            st, Xp, Up, _ = ffi.prologue(kp, cfgv, N, M, x[b], X[b], U[b], warm=int(step > 0))
            q = ffi.build_qp(kp, cfgv, N, M, Xp, Up)
            w0, k0 = ffi.qp_solve(q["H"], q["h"], q["lb"], q["ub"], q["C"], q["c"], K)
            E = np.random.default_rng(1000 * b + step).normal(size=q["H"].shape) * 1e-15
            w1, k1 = ffi.qp_solve(q["H"] * (1 + (E + E.T) / 2), q["h"], q["lb"], q["ub"], q["C"], q["c"], K)
            if k0 < 1e-10 and k1 < 1e-10:
                errs.append(np.abs(w1 - w0).max() / max(1.0, np.abs(w0).max()))
        ffi.rti_step(kp, cfgv, N, M, K, x, X, U, warm=int(step > 0), nthreads=0)
        x = X[:, 1, :].copy()
    e = np.array(errs)
    assert e.size >= 0.9 * B * 6
    assert e.max() < COND_ENVELOPE and np.median(e) < 1e-8, (e.max(), np.median(e))
    assert e.max() > 1e-9                              # the envelope is real: rounding moves solutions
    print(f"condensed QP envelope: {e.size} frozen solves, median {np.median(e):.1e}, max {e.max():.1e}")


def test_recursive_residuals_keep_the_iterations(kp):
    """The condensed IPM's recursive residuals (cfg qp_rec, k_qp_tiled's rule,
    DESIGN 4.3): along a closed loop, each step solved from the same inputs
    with exact residuals and with recursive ones above 1e-6 takes the same
    number of IPM iterations, and the committed steps agree within the QP's
    perturbation envelope (COND_ENVELOPE), the typical kite at rounding level."""
    from tests.test_gpu_parity import COND_ENVELOPE, x0_batch
    N, M, K, B = 20, 2, 16, 48
    base = dict(ffi.node_config(N=N), qp_form=0)
    cv_exact, cv_rec = ffi.cfg_vector(dict(base, qp_rec=0.0)), ffi.cfg_vector(dict(base, qp_rec=1e-6))
    assert ffi.cfg_vector(base)[132] == 1e-6                 # the N = 20 default is k_qp_tiled's rule
    x = x0_batch(B, offset=4100)
    X = np.zeros((B, N + 1, 15)); U = np.zeros((B, N, 4))
    d = []
    for step in range(5):
        Xr, Ur = X.copy(), U.copy()
        ie, ir = np.zeros(B, dtype=np.int32), np.zeros(B, dtype=np.int32)
        ffi.rti_step(kp, cv_exact, N, M, K, x, X, U, warm=int(step > 0), nthreads=8, iters=ie)
        ffi.rti_step(kp, cv_rec, N, M, K, x, Xr, Ur, warm=int(step > 0), nthreads=8, iters=ir)
        np.testing.assert_array_equal(ie, ir)
        d.append(np.maximum(np.abs(Xr - X).reshape(B, -1).max(1) / np.maximum(1, np.abs(X).reshape(B, -1).max(1)),
                            np.abs(Ur - U).reshape(B, -1).max(1) / np.maximum(1, np.abs(U).reshape(B, -1).max(1))))
        x = X[:, 1, :].copy()
    d = np.concatenate(d)
    assert d.max() < COND_ENVELOPE and np.median(d) < 1e-8, (d.max(), np.median(d))


def test_delay_compensation_prologue(kp):
    """Delay compensation (nmpf_node.cpp:206-221) in the oracle prologue: kite
    state predicted over 0.1 s under the previous u(t0) with 16 RK4 substeps,
    theta/thetadot from the previous trajectory at node round(0.1/0.05) = 2."""
    N, M = 20, 2
    c = ffi.node_config()
    c["delay"], c["delay_steps"] = 0.1, 16
    cv = ffi.cfg_vector(c)
    x0 = np.zeros(15)
    x0[:13] = ffi.synthetic_states(1, offset=5)[0]
    st, X, U, _ = ffi.prologue(kp, cv, N, M, x0, np.zeros((N + 1, 15)), np.zeros((N, 4)), warm=0)
    X[:, 13] += 0.3
    X[:, 14] += 1.7
    U[0, :3] = [0.12, 0.01, -0.02]
    st2, X2, U2, x0p = ffi.prologue(kp, cv, N, M, x0, X, U, warm=1)
    up = np.array([0.12, 0.01, -0.02, 0.0])
    pred = ffi.rk4(kp, x0, up, 0.1 / 16, 16)
    np.testing.assert_array_equal(x0p[:13], pred[:13])
    assert x0p[13] == X[2, 13] and x0p[14] == X[2, 14]
    np.testing.assert_array_equal(X2[0], x0p)
    # delay = 0: the measured state is used as given (KiteNMPF semantics)
    st3, _, _, x0q = ffi.prologue(kp, ffi.cfg_vector(ffi.node_config()), N, M, x0, X, U, warm=1)
    np.testing.assert_array_equal(x0q, x0)


def test_prologue_restarts_on_nonfinite_plan(kp, cfgv):
    """A NaN in the warm start (a failed previous iterate) restarts the kite
    cold: status bit 64, theta from the closest point, thetadot = 0."""
    N, M = 20, 2
    x0 = np.zeros(15)
    x0[:13] = ffi.synthetic_states(1, offset=8)[0]
    x0[13], x0[14] = np.nan, 3.0
    X = np.zeros((N + 1, 15)); U = np.zeros((N, 4))
    X[7, 2] = np.nan
    st, Xw, Uw, x0w = ffi.prologue(kp, cfgv, N, M, x0, X, U, warm=1)
    assert st & 64
    th = ffi.closest_point(cfgv, x0[6:9], 0.0)
    xc = x0.copy(); xc[13], xc[14] = th, 0.0
    st2, Xc, Uc, _ = ffi.prologue(kp, cfgv, N, M, xc, np.zeros((N + 1, 15)), np.zeros((N, 4)), warm=0)
    np.testing.assert_array_equal(Xw, Xc)
    np.testing.assert_array_equal(Uw, Uc)
    assert st2 & 64 == 0


MS_ENVELOPE = 3e-5   # the multiple-shooting QP's frozen-solution envelope (see below); the
                     # bar of tests/test_gpu_parity.py::assert_ms_rti for QPs frozen on both sides


def test_ms_qp_sensitivity_envelope(kp):
    """Intrinsic sensitivity of the multiple-shooting QP (qp_form 1, N = 40:
    BASELINE config 5) on closed-loop inputs: the QP data (A_k, B_k, d_k, J_k,
    r_k, R, rho) perturbed by a relative 1e-15 -- rounding-level differences
    between two fp64 implementations -- and solved again.  Where the perturbed
    IPM takes the same number of iterations the frozen solutions agree to
    ~1e-9; where it freezes one iteration earlier or later they move by up to
    ~1e-5 (tools/ms_envelope_probe.py 512 23 40: 5 of 23 512 perturbed solves,
    max 1.2e-5; same count: max 5.3e-9).  That sets assert_ms_rti's bar:
    MS_ENVELOPE for every QP frozen on both sides, RTI_TOL for >= 99.5 % of them."""
    from tests.test_gpu_parity import x0_batch
    Nh, M, K, B, steps = 40, 2, 16, 96, 8
    cv = ffi.cfg_vector(ffi.node_config(N=Nh))
    x = x0_batch(B, offset=11000)
    X = np.zeros((B, Nh + 1, 15)); U = np.zeros((B, Nh, 4))
    same, moved = [], []
    for step in range(steps):
        for b in range(B):
            st, Xp, Up, _ = ffi.prologue(kp, cv, Nh, M, x[b], X[b], U[b], warm=int(step > 0))
            v0, k0, i0 = ffi.msqp_solve(kp, cv, Nh, M, Xp, Up, K)
            v1, k1, i1 = ffi.msqp_solve_perturbed(kp, cv, Nh, M, Xp, Up, K, 1e-15, 1000 * b + step)
            if k0 < 1e-10 and k1 < 1e-10:
                e = np.abs(v1 - v0).max() / max(1.0, np.abs(v0).max())
                (same if i0 == i1 else moved).append(e)
        ffi.rti_step(kp, cv, Nh, M, K, x, X, U, warm=int(step > 0), nthreads=0)
        x = X[:, 1, :].copy()
    same, moved = np.array(same), np.array(moved)
    assert same.size + moved.size >= 0.99 * B * steps
    assert same.max() < 1e-7, same.max()
    assert moved.max(initial=0.0) < MS_ENVELOPE, moved
    assert np.mean(np.concatenate([same, moved]) < 1e-6) >= 0.995
    print(f"MS QP envelope: {same.size} same-count solves max {same.max():.1e}, "
          f"{moved.size} with a changed count max {moved.max(initial=0.0):.1e}")


@pytest.mark.parametrize("N", [20, 40])
def test_condensed_qp_is_the_eliminated_ms_qp(kp, N):
    """Two code paths of the oracle build the same QP: the condensed H, h of
    build_qp (condensing inside the RK4 sweep) equal the multiple-shooting
    data of build_msqp (A_k, B_k, d_k, residual rows J_k, r_k, control terms)
    condensed here in numpy, dx_{k+1} = A_k dx_k + B_k du_k + d_k eliminated,
    in the same scaled variables w = [du_0 .. du_{N-1}, dtheta_0,
    dthetadot_0].  Cold-start linearisation points of 4 synthetic kites."""
    c = ffi.node_config(N=N)
    cv = ffi.cfg_vector(c)
    xs = ffi.synthetic_states(4, offset=11000)
    nu, n = 4, 4 * N + 2
    for b in range(4):
        x0 = np.zeros(15); x0[:13] = xs[b]; x0[13] = ffi.closest_point(cv, xs[b, 6:9])
        _, Xp, Up, _ = ffi.prologue(kp, cv, N, 2, x0, np.zeros((N + 1, 15)), np.zeros((N, 4)), warm=0)
        q = ffi.build_qp(kp, cv, N, 2, Xp, Up)
        m = ffi.msqp_build(kp, cv, N, 2, Xp, Up)
        G = np.zeros((N + 1, 15, n)); g = np.zeros((N + 1, 15))
        G[0, 13, nu * N] = 1.0; G[0, 14, nu * N + 1] = 1.0
        for k in range(N):
            G[k + 1] = m["A"][k] @ G[k]
            G[k + 1][:, nu * k:nu * k + nu] += m["B"][k]
            g[k + 1] = m["A"][k] @ g[k] + m["d"][k]
        H = np.zeros((n, n)); h = np.zeros(n)
        for k in range(N + 1):
            nr = 4 if k < N else 3
            W = m["J"][k, :nr] @ G[k]
            H += W.T @ W
            h += W.T @ (m["r"][k, :nr] + m["J"][k, :nr] @ g[k])
            if k < N:
                H[nu * k:nu * k + nu, nu * k:nu * k + nu] += np.diag(m["Rh"])
                h[nu * k:nu * k + nu] += m["rho"][k]
        assert np.abs(H - q["H"]).max() <= 1e-12 * np.abs(q["H"]).max()
        assert np.abs(h - q["h"]).max() <= 1e-12 * np.abs(q["h"]).max()
