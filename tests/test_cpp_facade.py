"""The C++ KiteNMPF facade (include/kite_nmpc/KiteNMPF.hpp) driven the way the
reference ROS node drives KiteNMPF (tests/cpp/facade_main.cpp: every call of
nmpf_node.cpp).  CPU: it compiles and links against the C ABI, and the path
evaluator behind getPathFunction() matches the oracle.  GPU: its closed loop
equals, bitwise, the same sequence run through the Python binding."""
import ctypes
import json
import os
import subprocess

import numpy as np
import pytest

import openkite_amd as ok
from oracle import ffi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tests", "cpp", "facade_main.cpp")
LIBDIR = os.path.join(REPO, "openkite_amd", "lib")


def build(tmp_path):
    exe = str(tmp_path / "facade_main")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I", os.path.join(REPO, "include"), SRC,
                    "-L", LIBDIR, "-lkite_nmpc", f"-Wl,-rpath,{LIBDIR}", "-o", exe], check=True)
    return exe


def test_facade_compiles_and_links(tmp_path):
    assert os.path.exists(build(tmp_path))


def test_path_eval_matches_oracle(cfgv):
    """kite_nmpc_path_eval (getPathFunction, nmpf_node.cpp:30-40) vs the oracle path."""
    th = np.linspace(-7, 7, 57)
    P, dP = ok.path_eval(ok.default_config(), th)
    for i, t in enumerate(th):
        Po, dPo = ffi.path(cfgv, t)
        np.testing.assert_allclose(P[i], Po, rtol=0, atol=1e-15)
        np.testing.assert_allclose(dP[i], dPo, rtol=0, atol=1e-15)
    nm = ok.KiteNMPF()
    np.testing.assert_array_equal(nm.getPathFunction()(th[3]), P[3])


@pytest.mark.gpu
def test_facade_node_sequence_matches_python_binding(tmp_path):
    exe = build(tmp_path)
    steps = 4
    xs = ffi.synthetic_states(1, offset=77)[0]
    out = subprocess.run([exe, ok.nmpc.DEFAULT_PARAMS, str(steps)] + [repr(float(v)) for v in xs], check=True,
                         capture_output=True, text=True).stdout
    recs = [json.loads(l) for l in out.strip().splitlines()]
    assert len(recs) == steps
    g = ok.BatchNMPC(ok.load_properties(), ok.default_config(), 1)
    cfg = ok.default_config()
    N = cfg.N
    try:
        kite_state, control, traj, status = xs.copy(), np.zeros(3), None, None
        for r in recs:
            if traj is None:
                aug = np.r_[kite_state, g.closest_point(kite_state[6:9].reshape(1, 3), np.zeros(1))[0], 0.0]
                prev = "none"
            else:
                xp = g.predict(np.r_[kite_state, 0.0, 0.0].reshape(1, 15), np.r_[control, 0.0].reshape(1, 4), 0.1, 16)[0]
                aug = np.r_[xp[:13], traj[2, 13:15]]          # column N-2 of the reversed order = node 2
                prev = ok.nmpc._ReturnStatus(status).return_status
            aug[0] = max(aug[0], 2.1)
            res = g.step(aug.reshape(1, 15))
            traj, status = res["traj"][0], int(res["status"][0])
            control = res["u0"][0, :3]
            assert r["prev_status"] == prev
            assert r["ctrl_cols"] == N + 1 and r["traj_cols"] == N + 1
            np.testing.assert_array_equal(np.array(r["aug"]), aug)
            np.testing.assert_array_equal(np.array(r["control"]), control)
            np.testing.assert_array_equal(np.array(r["x1"]), traj[1])
            assert r["status"] == "Solve_Succeeded"
            assert r["pos_error"] == res["diag"][0, 0] and r["vel_error"] == res["diag"][0, 1]
            assert r["virt_state"] == traj[0, 13]
            np.testing.assert_array_equal(np.array(r["virt_t0"]), ok.path_eval(cfg, [traj[0, 13]])[0][0])
            np.testing.assert_array_equal(np.array(r["virt_tf"]), ok.path_eval(cfg, [traj[N, 13]])[0][0])
            kite_state = traj[1, :13].copy()
    finally:
        g.close()


def test_facade_fourier_path(tmp_path):
    """KiteNMPF(params, FourierPath) -> getPathFunction() equals the C ABI's
    path evaluator on the same Fourier path (the reference's KiteNMPF takes any
    path Function, kiteNMPF.h:14)."""
    from test_path import fourier_path, product_config
    exe = str(tmp_path / "facade_path")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "cpp", "facade_path.cpp"), "-L", LIBDIR, "-lkite_nmpc",
                    f"-Wl,-rpath,{LIBDIR}", "-o", exe], check=True)
    F = fourier_path()
    cfg = product_config(F)
    q = list(cfg.path_q)
    args = [repr(float(v)) for v in F.reshape(-1)] + [repr(float(v)) for v in q] + [ok.nmpc.DEFAULT_PARAMS]
    out = subprocess.run([exe] + args, check=True, capture_output=True, text=True).stdout.split("\n")
    rows = np.array([[float(t) for t in l.split()] for l in out if l.strip()])
    P, _ = ok.path_eval(cfg, rows[:, 0])
    np.testing.assert_array_equal(rows[:, 1:], P)
