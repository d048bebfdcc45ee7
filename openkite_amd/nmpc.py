"""Python host side of the MI355X kite NMPC: ctypes binding of the C ABI
(include/kite_nmpc/kite_nmpc.h) plus a ``KiteNMPF`` class that mirrors the
reference controller API (src/kite_control/kiteNMPF.h:10-118).

Every numerical call goes to libkite_nmpc.so on the GPU; if the library is
missing or no gfx950 device is present the calls raise -- there is no CPU
fallback.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KITE_NMPC_LIB", os.path.join(_HERE, "lib", "libkite_nmpc.so"))
REPO = os.path.dirname(_HERE)
DEFAULT_PARAMS = os.path.join(REPO, "data", "umx_radian.yaml")

KITE_OK, KITE_EINVAL, KITE_EHIP, KITE_ENOMEM, KITE_ENODEV, KITE_EIO, KITE_EPARSE, KITE_ESTATE = 0, -1, -2, -3, -4, -5, -6, -7
ST_NAN, ST_QP_NOT_CONV, ST_MIN_SPEED, ST_STATE_BOUND, ST_THETA_WRAP, ST_STEP_REJECTED = 1, 2, 4, 8, 16, 32
ST_RESTART = 64

_PARAM_FIELDS = ["b", "c", "AR", "S", "lam", "St", "lt", "Sf", "lf", "Xac",
                 "mass", "Ixx", "Iyy", "Izz", "Ixz",
                 "CL0", "CL0_tail", "CLa_total", "CLa_wing", "CLa_tail", "e_oswald",
                 "CD0_total", "CD0_wing", "CD0_tail", "CYb", "CYb_vtail", "Cm0", "Cma",
                 "Cn0", "Cnb", "Cl0", "Clb", "CLq", "Cmq", "CYr", "Cnr", "Clr", "CYp", "Clp", "Cnp",
                 "CLde", "CYdr", "Cmde", "Cndr", "Cldr", "CDde",
                 "Lt", "Ks", "Kd", "rx", "ry", "rz"]


class KiteParams(ctypes.Structure):
    """kite_params (KiteProperties flattened, kite.h:9-93)."""
    _fields_ = [(f, ctypes.c_double) for f in _PARAM_FIELDS]

    def as_array(self) -> np.ndarray:
        return np.array([getattr(self, f) for f in _PARAM_FIELDS], dtype=np.float64)


PATH_HMAX = 8                      # KITE_PATH_MAX_HARMONICS
PATH_NC = 2 * PATH_HMAX + 1


class NmpcConfig(ctypes.Structure):
    _fields_ = [
        ("N", ctypes.c_int32), ("M", ctypes.c_int32), ("qp_iters", ctypes.c_int32), ("shift", ctypes.c_int32),
        ("device", ctypes.c_int32), ("timing", ctypes.c_int32), ("qp_kernel", ctypes.c_int32),
        ("delay_steps", ctypes.c_int32),
        ("dt", ctypes.c_double), ("Q", ctypes.c_double * 3), ("R", ctypes.c_double * 4), ("W", ctypes.c_double),
        ("Sx", ctypes.c_double * 15), ("Su", ctypes.c_double * 4),
        ("lbx", ctypes.c_double * 15), ("ubx", ctypes.c_double * 15),
        ("lbu", ctypes.c_double * 4), ("ubu", ctypes.c_double * 4),
        ("vref", ctypes.c_double), ("path_radius", ctypes.c_double), ("path_altitude", ctypes.c_double),
        ("path_q", ctypes.c_double * 4), ("theta_flex", ctypes.c_double), ("min_speed", ctypes.c_double),
        ("delay", ctypes.c_double),
        ("sens_fp32", ctypes.c_int32), ("reserved", ctypes.c_int32),
        ("qp_soft_weight", ctypes.c_double), ("qp_lm", ctypes.c_double),
        ("path_harmonics", ctypes.c_int32), ("reserved2", ctypes.c_int32),
        ("path_fourier", ctypes.c_double * (3 * PATH_NC)),   # [3][2 * 8 + 1], row-major
    ]

    def set_fourier_path(self, coef, q=None) -> None:
        """Arbitrary closed path (KiteNMPF(kite, path), kiteNMPF.h:14): coef is
        (3, 2K + 1) per axis [c0, a1, b1, ..., aK, bK] of the unrotated curve
        p_a(theta) = c0 + sum_k a_k cos(k theta) + b_k sin(k theta), K <= 8;
        P = rot(q) p as for the circle (q None: keep path_q)."""
        c = np.asarray(coef, dtype=np.float64)
        if c.ndim != 2 or c.shape[0] != 3 or c.shape[1] % 2 != 1 or not 3 <= c.shape[1] <= PATH_NC:
            raise ValueError("coef must be (3, 2K+1) with 1 <= K <= %d" % PATH_HMAX)
        F = np.zeros((3, PATH_NC))
        F[:, :c.shape[1]] = c
        self.path_harmonics = (c.shape[1] - 1) // 2
        for i, v in enumerate(F.reshape(-1)):
            self.path_fourier[i] = v
        if q is not None:
            for i in range(4):
                self.path_q[i] = q[i]

    def to_dict(self) -> dict:
        d = {}
        for name, _ in self._fields_:
            v = getattr(self, name)
            d[name] = list(v) if hasattr(v, "__len__") else v
        return d


class CollocConfig(ctypes.Structure):
    """kite_colloc_config: the reference's collocation NLP functions (chebyshev.hpp)."""
    _fields_ = [
        ("poly_order", ctypes.c_int32), ("num_segments", ctypes.c_int32), ("use_R", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("t0", ctypes.c_double), ("tf", ctypes.c_double), ("Q", ctypes.c_double * 3), ("R", ctypes.c_double * 4),
        ("W", ctypes.c_double), ("vref", ctypes.c_double), ("mayer_scale", ctypes.c_double),
        ("Sx", ctypes.c_double * 15), ("Su", ctypes.c_double * 4),
        ("path_radius", ctypes.c_double), ("path_altitude", ctypes.c_double), ("path_q", ctypes.c_double * 4),
        ("path_harmonics", ctypes.c_int32), ("reserved2", ctypes.c_int32),
        ("path_fourier", ctypes.c_double * (3 * PATH_NC)),
    ]

    def to_dict(self) -> dict:
        d = {}
        for name, _ in self._fields_:
            v = getattr(self, name)
            d[name] = list(v) if hasattr(v, "__len__") else v
        return d


class MpcDiagnostic(ctypes.Structure):
    """msg/mpc_diagnostic.msg field order."""
    _fields_ = [("pos_error", ctypes.c_double), ("vel_error", ctypes.c_double), ("cost", ctypes.c_double),
                ("virt_state", ctypes.c_double), ("virt_ctrl", ctypes.c_double), ("comp_time_ms", ctypes.c_double)]


DIAG_FIELDS = [f for f, _ in MpcDiagnostic._fields_]

_lib = None
_DP = ctypes.POINTER(ctypes.c_double)
_IP = ctypes.POINTER(ctypes.c_int32)

# every symbol of include/kite_nmpc/kite_nmpc.h with its ctypes signature
_SIGNATURES = {
    "kite_nmpc_api_version": (ctypes.c_int, []),
    "kite_nmpc_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "kite_params_load_yaml": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(KiteParams)]),
    "kite_nmpc_default_config": (None, [ctypes.POINTER(NmpcConfig)]),
    "kite_nmpc_create": (ctypes.c_int, [ctypes.POINTER(KiteParams), ctypes.POINTER(NmpcConfig), ctypes.c_int32,
                                        ctypes.POINTER(ctypes.c_void_p)]),
    "kite_nmpc_destroy": (None, [ctypes.c_void_p]),
    "kite_nmpc_batch": (ctypes.c_int, [ctypes.c_void_p]),
    "kite_nmpc_set_bounds": (ctypes.c_int, [ctypes.c_void_p, _DP, _DP, _DP, _DP]),
    "kite_nmpc_set_reference_velocity": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_double]),
    "kite_nmpc_reset": (ctypes.c_int, [ctypes.c_void_p]),
    "kite_nmpc_set_wind": (ctypes.c_int, [ctypes.c_void_p, _DP]),
    "kite_nmpc_set_stream": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "kite_nmpc_use_own_stream": (ctypes.c_int, [ctypes.c_void_p]),
    "kite_nmpc_synchronize": (ctypes.c_int, [ctypes.c_void_p]),
    "kite_nmpc_closest_point": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, _DP, _DP, _DP]),
    "kite_nmpc_path_eval": (ctypes.c_int, [ctypes.POINTER(NmpcConfig), ctypes.c_int32, _DP, _DP, _DP]),
    "kite_nmpc_step": (ctypes.c_int, [ctypes.c_void_p, _DP, _DP, _DP, _DP, ctypes.POINTER(MpcDiagnostic), _IP]),
    "kite_nmpc_step_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "kite_nmpc_get_solution": (ctypes.c_int, [ctypes.c_void_p, _DP, _DP]),
    "kite_nmpc_set_solution": (ctypes.c_int, [ctypes.c_void_p, _DP, _DP]),
    "kite_nmpc_dynamics": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, _DP, _DP, _DP]),
    "kite_nmpc_jacobian": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, _DP, _DP, _DP, _DP]),
    "kite_nmpc_predict": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, _DP, _DP, ctypes.c_double,
                                         ctypes.c_int32, _DP]),
    "kite_nmpc_rk4_sens": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, _DP, _DP, ctypes.c_double,
                                          ctypes.c_int32, _DP, _DP, _DP]),
    "kite_nmpc_kernel_times": (ctypes.c_int, [ctypes.c_void_p, _DP, ctypes.c_int32]),
    "kite_nmpc_get_qp": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, _DP, _DP, _DP, _DP, _DP]),
    "kite_nmpc_timing_start": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32]),
    "kite_nmpc_timing_start_sampled": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]),
    "kite_nmpc_timing_read": (ctypes.c_int, [ctypes.c_void_p, _DP, ctypes.c_int32]),
    "kite_nmpc_qp_stats": (ctypes.c_int, [ctypes.c_void_p, _DP, _IP]),
    "kite_nmpc_qp_iteration_sum": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]),
    "kite_nmpc_state_bound_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64),
                                                   ctypes.POINTER(ctypes.c_int64)]),
    "kite_ekf_default_covariances": (None, [_DP, _DP, _DP]),
    "kite_colloc_default_config": (None, [ctypes.c_void_p]),
    "kite_nmpc_colloc_eval": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, _DP, _DP, _DP, _DP]),
    "kite_nmpc_ekf_step": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_double, _DP, _DP, _DP, _DP,
                                          _DP, _DP]),
    "kite_nmpc_ekf_step_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_double, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_void_p]),
}


class KiteNmpcError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        msg = lib().kite_nmpc_strerror(code).decode() if _lib is not None else str(code)
        super().__init__(f"{what}: {msg} ({code})" if what else f"{msg} ({code})")
        self.code = code


def lib():
    """Load libkite_nmpc.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: build it with `make -C openkite_amd/csrc` "
                               "(or __graft_entry__.build()); there is no CPU fallback")
        # One HIP runtime per process.  PyTorch-ROCm ships its own
        # libamdhip64 (SONAME libamdhip64.so.7) and NEEDs it by the unversioned
        # name: if /opt/rocm's copy is mapped first, torch maps a second one
        # and sees no GPU (and torch stream handles mean nothing to ours).
        # Mapping torch first makes our NEEDED libamdhip64.so.7 bind to it.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _check(code: int, what: str):
    if code < 0:
        raise KiteNmpcError(code, what)
    return code


def _p(a: Optional[np.ndarray]):
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"], "float64 C-contiguous array required"
    return a.ctypes.data_as(_DP)


def _f64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64)


def load_properties(path: str = DEFAULT_PARAMS) -> KiteParams:
    """kite_utils::LoadProperties (kite.cpp:7-76) via the C ABI."""
    p = KiteParams()
    _check(lib().kite_params_load_yaml(path.encode(), ctypes.byref(p)), f"load {path}")
    return p


def resolve_qp_kernel(qp_kernel: int, N: int) -> int:
    """The QP kernel a config selects (kite_nmpc_create): 0 (auto) is the
    register-tiled condensed QP (2) at N == 20, the multiple-shooting QP (3)
    otherwise."""
    return qp_kernel if qp_kernel else (2 if N == 20 else 3)


def default_config(**overrides) -> NmpcConfig:
    """The reference node's controller setup (nmpf_node.cpp:30-69) + RTI defaults."""
    c = NmpcConfig()
    lib().kite_nmpc_default_config(ctypes.byref(c))
    for k, v in overrides.items():
        if not hasattr(c, k):
            raise KeyError(k)
        cur = getattr(c, k)
        if hasattr(cur, "__len__"):
            for i, vi in enumerate(v):
                cur[i] = vi
        else:
            setattr(c, k, v)
    return c


class BatchNMPC:
    """A batch of independent NMPC instances on one GPU (one C-ABI context)."""

    def __init__(self, params: Optional[KiteParams] = None, config: Optional[NmpcConfig] = None,
                 batch: int = 1):
        self.params = params if params is not None else load_properties()
        self.config = config if config is not None else default_config()
        self.batch = int(batch)
        self.N = int(self.config.N)
        h = ctypes.c_void_p()
        _check(lib().kite_nmpc_create(ctypes.byref(self.params), ctypes.byref(self.config), self.batch,
                                      ctypes.byref(h)), "kite_nmpc_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().kite_nmpc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    # --- configuration ----------------------------------------------------
    def set_bounds(self, lbx=None, ubx=None, lbu=None, ubu=None):
        args = [None if a is None else _f64(a) for a in (lbx, ubx, lbu, ubu)]
        _check(lib().kite_nmpc_set_bounds(self._h, *[_p(a) for a in args]), "set_bounds")

    def set_reference_velocity(self, v: float):
        _check(lib().kite_nmpc_set_reference_velocity(self._h, float(v)), "set_reference_velocity")

    def reset(self):
        _check(lib().kite_nmpc_reset(self._h), "reset")

    def set_wind(self, wind=None):
        """Per-kite constant world-frame wind, (B, 3) m/s, for wind-field sweeps
        (kite_nmpc_set_wind; None or all zero = the reference model, which has
        no wind)."""
        if wind is None:
            _check(lib().kite_nmpc_set_wind(self._h, None), "set_wind")
            return
        w = np.ascontiguousarray(np.asarray(wind, dtype=np.float64).reshape(self.batch, 3))
        _check(lib().kite_nmpc_set_wind(self._h, w.ctypes.data_as(_DP)), "set_wind")

    def set_stream(self, stream_ptr: int):
        """Run on this hipStream_t (int handle; 0 = the HIP null stream, which is
        torch's default stream)."""
        _check(lib().kite_nmpc_set_stream(self._h, ctypes.c_void_p(stream_ptr) if stream_ptr else None),
               "set_stream")

    def use_own_stream(self):
        _check(lib().kite_nmpc_use_own_stream(self._h), "use_own_stream")

    def synchronize(self):
        _check(lib().kite_nmpc_synchronize(self._h), "synchronize")

    # --- RTI step -------------------------------------------------------------
    def step(self, x0: np.ndarray, want_traj: bool = True):
        B, N = self.batch, self.N
        x0 = _f64(x0).reshape(B, 15)
        u0 = np.zeros((B, 4))
        traj = np.zeros((B, N + 1, 15)) if want_traj else None
        ctrl = np.zeros((B, N, 4)) if want_traj else None
        diag = (MpcDiagnostic * B)()
        status = np.zeros(B, dtype=np.int32)
        _check(lib().kite_nmpc_step(self._h, _p(x0), _p(u0), _p(traj), _p(ctrl), diag,
                                    status.ctypes.data_as(_IP)), "kite_nmpc_step")
        d = np.ctypeslib.as_array(ctypes.cast(diag, _DP), shape=(B, 6)).copy()
        return dict(u0=u0, traj=traj, ctrl=ctrl, diag=d, status=status)

    def step_device(self, x0_ptr: int, u0_ptr=0, traj_ptr=0, ctrl_ptr=0, diag_ptr=0, status_ptr=0):
        v = lambda p: ctypes.c_void_p(p) if p else None
        _check(lib().kite_nmpc_step_device(self._h, v(x0_ptr), v(u0_ptr), v(traj_ptr), v(ctrl_ptr),
                                           v(diag_ptr), v(status_ptr)), "kite_nmpc_step_device")

    def get_solution(self):
        traj = np.zeros((self.batch, self.N + 1, 15)); ctrl = np.zeros((self.batch, self.N, 4))
        _check(lib().kite_nmpc_get_solution(self._h, _p(traj), _p(ctrl)), "get_solution")
        return traj, ctrl

    def set_solution(self, traj, ctrl):
        _check(lib().kite_nmpc_set_solution(self._h, _p(_f64(traj)), _p(_f64(ctrl))), "set_solution")

    TIMING_KEYS = ("prologue", "rk4_sens", "condense", "qp", "total", "qp_main")

    def kernel_times(self):
        """Device time [ms] of the last step per phase (config.timing = 1);
        qp is the QP phase (solve + expansion + lazy rows), qp_main the main
        QP kernel alone."""
        ms = np.zeros(6)
        n = _check(lib().kite_nmpc_kernel_times(self._h, _p(ms), 6), "kernel_times")
        return dict(zip(self.TIMING_KEYS, ms[:n]))

    def timing_start(self, max_steps: int, stride: int = 1):
        """Record the kernel events of every stride-th step from the next one
        on, at most max_steps of them (kite_nmpc_timing_start_sampled)."""
        if stride == 1:
            _check(lib().kite_nmpc_timing_start(self._h, int(max_steps)), "timing_start")
        else:
            _check(lib().kite_nmpc_timing_start_sampled(self._h, int(max_steps), int(stride)), "timing_start")

    def timing_read(self):
        """Per-phase SUMS [ms] over the steps recorded since timing_start
        (keys as kernel_times)."""
        ms = np.zeros(6)
        n = _check(lib().kite_nmpc_timing_read(self._h, _p(ms), 6), "timing_read")
        return n, dict(zip(self.TIMING_KEYS, ms))

    def qp_stats(self):
        kkt = np.zeros(self.batch); it = np.zeros(self.batch, dtype=np.int32)
        _check(lib().kite_nmpc_qp_stats(self._h, _p(kkt), it.ctypes.data_as(_IP)), "qp_stats")
        return kkt, it

    def qp_iteration_sum(self) -> int:
        """QP iterations summed over instances and steps since timing_start."""
        v = ctypes.c_int64(0)
        _check(lib().kite_nmpc_qp_iteration_sum(self._h, ctypes.byref(v)), "qp_iteration_sum")
        return int(v.value)

    def state_bound_stats(self):
        """(kite-steps outside the state box, (node, state) pairs outside it),
        summed over instances and steps since timing_start (status bit 8 and
        the violated state rows of the committed plans)."""
        a, r = ctypes.c_int64(0), ctypes.c_int64(0)
        _check(lib().kite_nmpc_state_bound_stats(self._h, ctypes.byref(a), ctypes.byref(r)), "state_bound_stats")
        return int(a.value), int(r.value)

    def get_qp(self, instance: int):
        n = 4 * self.N + 2
        H = np.zeros((n, n)); h = np.zeros(n); C = np.zeros((self.N, n)); cl = np.zeros(self.N); cu = np.zeros(self.N)
        _check(lib().kite_nmpc_get_qp(self._h, int(instance), _p(H), _p(h), _p(C), _p(cl), _p(cu)), "get_qp")
        return dict(H=H, h=h, C=C, cl=cl, cu=cu)

    # --- model-level ----------------------------------------------------------
    def closest_point(self, pos, guess=None):
        pos = _f64(pos).reshape(-1, 3)
        out = np.zeros(pos.shape[0])
        g = None if guess is None else _f64(guess).reshape(-1)
        _check(lib().kite_nmpc_closest_point(self._h, pos.shape[0], _p(pos), _p(g), _p(out)), "closest_point")
        return out

    def dynamics(self, x15, u4):
        x = _f64(x15).reshape(-1, 15); u = _f64(u4).reshape(-1, 4)
        f = np.zeros_like(x)
        _check(lib().kite_nmpc_dynamics(self._h, x.shape[0], _p(x), _p(u), _p(f)), "dynamics")
        return f

    def jacobian(self, x13, u3):
        x = _f64(x13).reshape(-1, 13); u = _f64(u3).reshape(-1, 3)
        Jx = np.zeros((x.shape[0], 13, 13)); Ju = np.zeros((x.shape[0], 13, 3))
        _check(lib().kite_nmpc_jacobian(self._h, x.shape[0], _p(x), _p(u), _p(Jx), _p(Ju)), "jacobian")
        return Jx, Ju

    def colloc_eval(self, cfg: "CollocConfig", z, jac: bool = False):
        """Reference collocation residual G (count x n*15), cost J (count) and,
        with jac, the per-node blocks d SODE / d [x, u] (count x n x 15 x 19)."""
        n = cfg.poly_order * cfg.num_segments + 1
        zz = _f64(z).reshape(-1, n * 19)
        c = zz.shape[0]
        G = np.zeros((c, n * 15)); J = np.zeros(c)
        Jb = np.zeros((c, n, 15, 19)) if jac else None
        _check(lib().kite_nmpc_colloc_eval(self._h, ctypes.byref(cfg), c, _p(zz), _p(G), _p(J), _p(Jb)), "colloc_eval")
        return (G, J, Jb) if jac else (G, J)

    def ekf_step_device(self, count: int, dt: float, d_x13: int, d_u3: int, d_P169: int, d_z7: int,
                        d_W169: int, d_V49: int):
        """Device-pointer EKF step (asynchronous on the context stream)."""
        _check(lib().kite_nmpc_ekf_step_device(self._h, int(count), float(dt), d_x13, d_u3, d_P169, d_z7 or None,
                                               d_W169, d_V49), "ekf_step_device")

    def ekf_step(self, x13, u3, P, dt: float, z7=None, W=None, V=None):
        """Batched KiteEKF propagate (+ update when z7 is given); returns (x, P)."""
        x = _f64(x13).reshape(-1, 13).copy()
        c = x.shape[0]
        Pm = _f64(P).reshape(c, 13, 13).copy()
        u = _f64(u3).reshape(c, 3)
        Wd, Vd, _ = ekf_default_covariances()
        W = Wd if W is None else _f64(W).reshape(13, 13)
        V = Vd if V is None else _f64(V).reshape(7, 7)
        z = None if z7 is None else _f64(z7).reshape(c, 7)
        _check(lib().kite_nmpc_ekf_step(self._h, c, float(dt), _p(x), _p(u), _p(Pm), _p(z), _p(W), _p(V)),
               "ekf_step")
        return x, Pm

    def predict(self, x15, u4, tf: float, steps: int = 1):
        x = _f64(x15).reshape(-1, 15); u = _f64(u4).reshape(-1, 4)
        xo = np.zeros_like(x)
        _check(lib().kite_nmpc_predict(self._h, x.shape[0], _p(x), _p(u), float(tf), int(steps), _p(xo)), "predict")
        return xo

    def rk4_sens(self, x15, u4, tf: float, M: int):
        x = _f64(x15).reshape(-1, 15); u = _f64(u4).reshape(-1, 4)
        c = x.shape[0]
        xo = np.zeros((c, 15)); A = np.zeros((c, 15, 15)); Bm = np.zeros((c, 15, 4))
        _check(lib().kite_nmpc_rk4_sens(self._h, c, _p(x), _p(u), float(tf), int(M), _p(xo), _p(A), _p(Bm)),
               "rk4_sens")
        return xo, A, Bm


@dataclass
class _ReturnStatus:
    status: int

    @property
    def return_status(self) -> str:
        if self.status & ST_NAN:
            return "Invalid_Number_Detected"
        if self.status & ST_STEP_REJECTED:
            return "Restoration_Failed"
        if self.status & ST_QP_NOT_CONV:
            return "Maximum_Iterations_Exceeded"
        return "Solve_Succeeded"


def path_eval(config: NmpcConfig, theta):
    """P(theta) and dP/dtheta of the configured path (kite_nmpc_path_eval:
    getPathFunction, nmpf_node.cpp:30-40); host arithmetic, no GPU."""
    th = _f64(theta).reshape(-1)
    P = np.zeros((th.size, 3)); dP = np.zeros((th.size, 3))
    _check(lib().kite_nmpc_path_eval(ctypes.byref(config), th.size, _p(th), _p(P), _p(dP)), "path_eval")
    return P, dP


def colloc_default_config(**overrides) -> CollocConfig:
    """The NMPF's collocation setup (kiteNMPF.cpp:80-143 + node scaling/path)."""
    c = CollocConfig()
    lib().kite_colloc_default_config(ctypes.byref(c))
    for k, v in overrides.items():
        cur = getattr(c, k)
        if hasattr(cur, "__len__"):
            for i, vi in enumerate(v):
                cur[i] = vi
        else:
            setattr(c, k, v)
    return c


def ekf_default_covariances():
    """(W, V, P0) of KiteEKF (kiteEKF.cpp:6-13, P0 = 10 W at :26)."""
    W = np.zeros((13, 13)); V = np.zeros((7, 7)); P0 = np.zeros((13, 13))
    lib().kite_ekf_default_covariances(_p(W), _p(V), _p(P0))
    return W, V, P0


class KiteEKF:
    """Mirror of the reference ``KiteEKF`` (kiteEKF.h:10-55) for a batch of
    kites on one GPU context: same setters/getters, ``propagate(dt)`` and
    ``_estimate(measurement, dt)``; ``estimate(measurement, tstamp)`` takes
    dt = tstamp - getTimeStamp() and, as in the reference (kiteEKF.cpp:100-105),
    leaves the time stamp to ``setTime``."""

    def __init__(self, batch: int = 1, params: Optional[KiteParams] = None, device: int = 0):
        self._ctx = BatchNMPC(params if params is not None else load_properties(), default_config(device=device), batch)
        self.batch = batch
        self.W, self.V, P0 = ekf_default_covariances()
        self.P = np.repeat(P0[None], batch, axis=0)
        self.x = np.zeros((batch, 13))
        self.u = np.zeros((batch, 3))
        self.tstamp = 0.0

    def close(self):
        self._ctx.close()

    def setProcessCovariance(self, W): self.W = _f64(W).reshape(13, 13).copy()
    def setMeasurementCovariance(self, V): self.V = _f64(V).reshape(7, 7).copy()
    def setEstimationCovariance(self, P): self.P = np.broadcast_to(_f64(P).reshape(-1, 13, 13), (self.batch, 13, 13)).copy()
    def setEstimation(self, x): self.x = np.broadcast_to(_f64(x).reshape(-1, 13), (self.batch, 13)).copy()
    def setControl(self, u): self.u = np.broadcast_to(_f64(u).reshape(-1, 3), (self.batch, 3)).copy()
    def setTime(self, t): self.tstamp = float(t)
    def getEstimation(self): return self.x.copy()
    def getEstimationCovariance(self): return self.P.copy()
    def getTimeStamp(self): return self.tstamp

    def propagate(self, dt: float):
        self.x, self.P = self._ctx.ekf_step(self.x, self.u, self.P, dt, None, self.W, self.V)

    def _estimate(self, measurement, dt: float):
        z = np.broadcast_to(_f64(measurement).reshape(-1, 7), (self.batch, 7))
        self.x, self.P = self._ctx.ekf_step(self.x, self.u, self.P, dt, z, self.W, self.V)

    def estimate(self, measurement, tstamp: float):
        self._estimate(measurement, tstamp - self.tstamp)


class KiteNMPF:
    """Mirror of the reference ``KiteNMPF`` (kiteNMPF.h:10-118) for one kite.

    Setters / getters keep the reference names and semantics: matrices are
    returned in the reference's column order, i.e. time runs backwards and the
    LAST column of getOptimalControl() is u(t0) (nmpf_node.cpp:124).  The
    scaling matrices are diagonal; setReferenceVelocity is physical and, as
    in the reference, must be called after setStateScaling (it is stored in
    physical units here so the order no longer matters).
    """

    def __init__(self, params: Optional[KiteParams] = None, N: int = 20, dt: float = 0.05, **cfg):
        self._cfg = default_config(N=N, dt=dt, **cfg)
        self._params = params if params is not None else load_properties()
        self._impl: Optional[BatchNMPC] = None
        self._traj = None
        self._ctrl = None
        self._diag = None
        self._status = 0
        self._warm = False

    # setters kiteNMPF.h:20-34
    def setLBX(self, v): self._set("lbx", v)
    def setUBX(self, v): self._set("ubx", v)
    def setLBU(self, v): self._set("lbu", v)
    def setUBU(self, v): self._set("ubu", v)
    def setLBG(self, v): pass          # collocation equality bounds: no counterpart in the RTI
    def setUBG(self, v): pass

    def setStateScaling(self, S):
        self._set("Sx", np.diag(np.asarray(S, dtype=float)) if np.ndim(S) == 2 else S)

    def setControlScaling(self, S):
        self._set("Su", np.diag(np.asarray(S, dtype=float)) if np.ndim(S) == 2 else S)

    def setReferenceVelocity(self, v):
        self._cfg.vref = float(np.asarray(v).reshape(-1)[0])
        if self._impl is not None:
            self._impl.set_reference_velocity(self._cfg.vref)

    def setPath(self, radius: float, altitude: float = 0.0, q=(1.0, 0.0, 0.0, 0.0)):
        """The reference declares setPath(SX) but never defines it (kiteNMPF.h:36);
        the rotated circle of nmpf_node.cpp:30-40."""
        self._cfg.path_radius = radius
        self._cfg.path_altitude = altitude
        for i in range(4):
            self._cfg.path_q[i] = q[i]
        self._cfg.path_harmonics = 0
        self._impl = None

    def setPathFourier(self, coef, q=(1.0, 0.0, 0.0, 0.0)):
        """Any closed path (the path Function of KiteNMPF's ctor, kiteNMPF.h:14)
        as a rotated Fourier curve, see NmpcConfig.set_fourier_path."""
        self._cfg.set_fourier_path(coef, q)
        self._impl = None

    def _set(self, name, v):
        arr = getattr(self._cfg, name)
        for i, vi in enumerate(np.asarray(v, dtype=float).reshape(-1)):
            arr[i] = vi
        if self._impl is not None and name in ("lbx", "ubx", "lbu", "ubu"):
            self._impl.set_bounds(np.array(self._cfg.lbx), np.array(self._cfg.ubx),
                                  np.array(self._cfg.lbu), np.array(self._cfg.ubu))
        elif self._impl is not None:
            self._impl = None

    def createNLP(self):
        self._impl = BatchNMPC(self._params, self._cfg, 1)
        self._warm = False

    def enableWarmStart(self):
        self._warm = True

    def disableWarmStart(self):
        self._warm = False
        if self._impl is not None:
            self._impl.reset()

    def computeControl(self, X0):
        """KiteNMPF::computeControl (kiteNMPF.cpp:199-316) as one RTI step."""
        if self._impl is None:
            self.createNLP()
        if not self._warm:
            self._impl.reset()
        r = self._impl.step(np.asarray(X0, dtype=float).reshape(1, 15))
        self._traj, self._ctrl, self._diag, self._status = r["traj"][0], r["ctrl"][0], r["diag"][0], int(r["status"][0])
        self.enableWarmStart()

    def getOptimalControl(self):
        """4 x (N+1), reference shape and column order: column N - k = u_k (last
        column = u(t0)); column 0 (t = tf, where no interval starts) repeats
        u_{N-1}, the control held up to tf."""
        if self._ctrl is None:
            return None
        return np.vstack([self._ctrl, self._ctrl[-1:]])[::-1].T.copy()

    def getOptimalTrajetory(self):   # [sic] kiteNMPF.h:44
        """15 x (N+1), reference column order (last column = x(t0))."""
        return None if self._traj is None else self._traj[::-1].T.copy()

    def getPathFunction(self):
        """theta -> P(theta) (3,) of the configured path (kiteNMPF.h:46)."""
        cfg = self._cfg
        return lambda theta: path_eval(cfg, [theta])[0][0]

    def getStats(self):
        return {"return_status": _ReturnStatus(self._status).return_status, "status_bits": self._status}

    def getPathError(self):
        return 0.0 if self._diag is None else float(self._diag[0])

    def getVelocityError(self):
        return 0.0 if self._diag is None else float(self._diag[1])

    def getVirtState(self):
        return 0.0 if self._diag is None else float(self._diag[3])

    def initialized(self):
        return False   # never set true in the reference (kiteNMPF.cpp:46)

    def findClosestPointOnPath(self, position, init_guess=0.0):
        if self._impl is None:
            self.createNLP()
        return float(self._impl.closest_point(np.asarray(position, dtype=float).reshape(1, 3),
                                              np.array([float(init_guess)]))[0])

    def diagnostic(self):
        """mpc_diagnostic record (nmpf_node.cpp:191-204)."""
        return None if self._diag is None else dict(zip(DIAG_FIELDS, map(float, self._diag)))
