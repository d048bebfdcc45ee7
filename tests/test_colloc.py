"""The reference formulation evaluator: Chebyshev collocation
residual, cost and Jacobian of the NLP (chebyshev.hpp:241-333,
kiteNMPF.cpp:80-143).  Input pin: the 209-vector of kite_control_test.cpp:582-598
(tests/golden/colloc_full_generics.json; the reference test prints the
constraint Jacobian there and asserts nothing, so outputs are pinned through
the golden Chebyshev D / weights and the golden f, J of the model)."""
import json
import os

import numpy as np
import pytest

import openkite_amd as ok
from oracle import ffi

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "colloc_full_generics.json")))


def nmpf_cfg():
    return ok.colloc_default_config().to_dict()


def nmpf_points(B, seed=5):
    """Scaled NMPF NLP points around the in-flight state (11 nodes)."""
    c = nmpf_cfg()
    n = c["poly_order"] * c["num_segments"] + 1
    rng = np.random.default_rng(seed)
    xs = ffi.synthetic_states(B * n, offset=300).reshape(B, n, 13)
    X = np.zeros((B, n, 15)); X[:, :, :13] = xs
    X[:, :, 13] = rng.uniform(-3, 3, (B, n)); X[:, :, 14] = rng.uniform(0, 4, (B, n))
    U = np.column_stack([rng.uniform(0.1, 0.15, B * n), rng.uniform(-0.1, 0.1, (B * n, 2)),
                         rng.uniform(-5, 5, B * n)]).reshape(B, n, 4)
    X *= np.array(c["Sx"]); U *= np.array(c["Su"])
    return np.concatenate([X.reshape(B, -1), U.reshape(B, -1)], axis=1)


def dense_jacobian(c, blocks):
    """dG/dz from the per-node blocks: CompDiff (x) I - t_scale blockdiag."""
    P, S = c["poly_order"], c["num_segments"]
    n = P * S + 1
    CD = ffi.cheb_compD(P, S)
    ts = (c["tf"] - c["t0"]) / (2 * S)
    Jx = np.kron(CD, np.eye(15))
    Ju = np.zeros((n * 15, n * 4))
    for i in range(n):
        Jx[i * 15:(i + 1) * 15, i * 15:(i + 1) * 15] -= ts * blocks[i][:, :15]
        Ju[i * 15:(i + 1) * 15, i * 4:(i + 1) * 4] = -ts * blocks[i][:, 15:]
    return np.hstack([Jx, Ju])


GOLD = json.load(open(os.path.join(HERE, "golden", "kite_golden.json")))["colloc"]
COLLOC_TOL = 1e-12      # relative to max |G| and to J; the 50-digit golden is exact to fp64


def test_oracle_colloc_vs_golden(kp):
    """The oracle's collocation residual and cost at the reference test's own
    NLP point against an independent 50-digit restatement of
    CollocateDynamics / CollocateCost (tests/golden/gen_golden.py 'colloc')."""
    G, J = ffi.colloc_eval(kp, FIX["config"], np.array(FIX["z"]))
    g = np.array(GOLD["G"])
    assert np.abs(G[0] - g).max() <= COLLOC_TOL * np.abs(g).max()
    assert abs(J[0] - GOLD["J"]) <= COLLOC_TOL * abs(GOLD["J"])


@pytest.mark.gpu
def test_gpu_colloc_vs_golden():
    """The same golden on the GPU evaluator (k_colloc)."""
    c = FIX["config"]
    cfg = ok.colloc_default_config(**{k: v for k, v in c.items() if k != "lines"})
    g = ok.BatchNMPC(ok.load_properties(), ok.default_config(), 1)
    try:
        G, J, _ = g.colloc_eval(cfg, np.array(FIX["z"])[None], jac=True)
    finally:
        g.close()
    gg = np.array(GOLD["G"])
    assert np.abs(G[0] - gg).max() <= COLLOC_TOL * np.abs(gg).max()
    assert abs(J[0] - GOLD["J"]) <= COLLOC_TOL * abs(GOLD["J"])


def test_fixture_is_the_reference_vector():
    z = np.array(FIX["z"])
    assert z.size == 209 and z[0] == 0.322159 and z[-1] == -1.83182


@pytest.mark.parametrize("which", ["full_generics", "nmpf"])
def test_oracle_jacobian_vs_finite_differences(kp, which):
    c = FIX["config"] if which == "full_generics" else nmpf_cfg()
    z = np.array(FIX["z"]) if which == "full_generics" else nmpf_points(1)[0]
    G, J, Jb = ffi.colloc_eval(kp, c, z, jac=True)
    assert np.all(np.isfinite(G)) and np.isfinite(J[0]) and J[0] >= 0
    D = dense_jacobian(c, Jb[0])
    h = 1e-6
    for col in range(0, z.size, 7):
        zp = z.copy(); zp[col] += h
        zm = z.copy(); zm[col] -= h
        fd = (ffi.colloc_eval(kp, c, zp)[0][0] - ffi.colloc_eval(kp, c, zm)[0][0]) / (2 * h)
        np.testing.assert_allclose(D[:, col], fd, rtol=1e-6, atol=1e-6 * max(1.0, np.abs(fd).max()))


def test_oracle_residual_of_a_linear_trajectory(kp):
    """CompDiff differentiates exactly a trajectory linear in the CGL time tau
    (node 0 = tau +1 of segment 0; segment k spans tau + 2(S-1-k)), so
    G_i + t_scale * SODE(X_i, U_i) equals the slope at every node."""
    c = nmpf_cfg()
    P, S = c["poly_order"], c["num_segments"]
    n = P * S + 1
    z = nmpf_points(1)[0]
    s = np.array([np.cos((j - min(j // P, S - 1) * P) * np.pi / P) + 2 * (S - 1 - min(j // P, S - 1))
                  for j in range(n)])
    slope = np.linspace(0.1, 1.5, 15)
    X = z[:15] + np.outer(s, slope)
    U = z[n * 15:].reshape(n, 4)
    G = ffi.colloc_eval(kp, c, np.r_[X.reshape(-1), U.reshape(-1)])[0][0].reshape(n, 15)
    Sx, Su = np.array(c["Sx"]), np.array(c["Su"])
    ts = (c["tf"] - c["t0"]) / (2 * S)
    sode = np.array([Sx * ffi.rhs_aug(kp, X[i] / Sx, U[i] / Su) for i in range(n)])
    np.testing.assert_allclose(G + ts * sode, np.tile(slope, (n, 1)), rtol=1e-11, atol=1e-11)


def fourier_colloc_cfg():
    """The NMPF setup on the three-harmonic path of tests/test_path.py."""
    from test_path import fourier_path
    F = np.zeros((3, 17)); F[:, :7] = fourier_path()
    cfg = ok.colloc_default_config()
    cfg.path_harmonics = 3
    for i, v in enumerate(F.reshape(-1)):
        cfg.path_fourier[i] = v
    return cfg


def test_oracle_colloc_circle_as_fourier(kp):
    """The collocation cost on the node's circle written as a K = 1 Fourier
    curve equals the circle's (oracle); a non-circular path changes it."""
    c0 = nmpf_cfg()
    c1 = dict(c0, path_harmonics=1)
    F = np.zeros((3, 17)); F[0, 1] = c0["path_radius"]; F[1, 2] = c0["path_radius"]; F[2, 0] = c0["path_altitude"]
    c1["path_fourier"] = F.reshape(-1)
    z = nmpf_points(16)
    G0, J0 = ffi.colloc_eval(kp, c0, z)
    G1, J1 = ffi.colloc_eval(kp, c1, z)
    np.testing.assert_array_equal(G0, G1)
    np.testing.assert_allclose(J0, J1, rtol=1e-14)
    _, J2 = ffi.colloc_eval(kp, fourier_colloc_cfg().to_dict(), z)
    assert np.abs(J2 - J0).max() > 1e-3 * np.abs(J0).max()


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["full_generics", "nmpf", "nmpf_fourier"])
def test_gpu_colloc_vs_oracle(kp, which):
    if which == "full_generics":
        c = FIX["config"]
        z = np.array(FIX["z"])[None]
        cfg = ok.colloc_default_config(**{k: v for k, v in c.items() if k != "lines"})
    elif which == "nmpf":
        c = nmpf_cfg()
        z = nmpf_points(512)
        cfg = ok.colloc_default_config()
    else:
        cfg = fourier_colloc_cfg()
        c = cfg.to_dict()
        z = nmpf_points(512)
    g = ok.BatchNMPC(ok.load_properties(), ok.default_config(), 1)
    try:
        G, J, Jb = g.colloc_eval(cfg, z, jac=True)
    finally:
        g.close()
    Go, Jo, Jbo = ffi.colloc_eval(kp, c, z, jac=True)
    np.testing.assert_allclose(G, Go, rtol=1e-12, atol=1e-12 * np.abs(Go).max())
    np.testing.assert_allclose(J, Jo, rtol=1e-12)
    np.testing.assert_allclose(Jb, Jbo, rtol=1e-12, atol=1e-12 * np.abs(Jbo).max())
