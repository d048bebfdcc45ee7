"""Per-rank closed-loop fleet driver: the loop bench.py times on every GPU.

One step of a fleet of kites on one rank:

  [EKF]  estimator (kiteEKF.cpp:75-126, BASELINE configs[4]): propagate the
         estimate under the control applied last, in `ekf_substeps` RK4 steps
         of dt/ekf_substeps, and update it with the measured position +
         attitude (z, 7 values) on the last one; the RTI starts from the
         estimate.
  RTI    one real-time iteration of the NMPC for every kite of the shard
         (kite_nmpc_step_device: KiteNMPF::computeControl, kiteNMPF.cpp:199-316).
  pub    optional publish of u0 + mpc_diagnostic of every kite to every rank
         (shard.Publisher: one all-gather, RCCL over xGMI / gloo on CPU).
  plant  closed loop on synthetic data: the next measured state is the plan's
         prediction at t0 + dt (trajectory node 1), and its position +
         attitude are the next EKF measurement.  With ``noise`` (a
         ``MeasurementNoise``) that state is disturbed before it is measured:
         the controller's model no longer predicts the plant exactly.

The stepper does the arithmetic; ``GpuStepper`` drives libkite_nmpc.so on
device tensors.  Tests plug a CPU oracle stepper into the same loop to check
the sharded multi-rank flow against the unsharded batch.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch


class GpuStepper:
    """RTI + EKF of one C-ABI context on device tensors (asynchronous on the
    context stream; give the context torch's stream with ``set_stream``)."""

    def __init__(self, ctx):
        self.ctx = ctx

    def rti(self, x0, u0, traj, diag, status):
        self.ctx.step_device(x0.data_ptr(), u0.data_ptr(), traj.data_ptr(), 0, diag.data_ptr(),
                             status.data_ptr())

    def ekf(self, dt, xe, u3, P, z, W, V):
        self.ctx.ekf_step_device(xe.shape[0], dt, xe.data_ptr(), u3.data_ptr(), P.data_ptr(),
                                 z.data_ptr() if z is not None else 0, W.data_ptr(), V.data_ptr())


class MeasurementNoise:
    """Seeded Gaussian disturbance of the measured kite state (bench.py
    --meas-noise): per step and kite, body velocity += 0.05 S, body rates +=
    0.05 S, position += 0.01 S (N(0, 1) draws, SI units), attitude rotated by
    a random small angle of about 0.01 S rad (quaternion renormalised);
    theta / thetadot are the controller's own states and stay untouched.  The
    draws come from a device generator seeded per rank, so a run is
    reproducible and the noise costs two small kernels per step."""

    SCALE = (0.05, 0.05, 0.01, 0.005)

    def __init__(self, sigma: float, device, seed: int):
        self.sigma = float(sigma)
        self.gen = torch.Generator(device=device)
        self.gen.manual_seed(int(seed))

    def apply(self, x: torch.Tensor) -> None:
        B = x.shape[0]
        n = torch.randn((B, 13), generator=self.gen, dtype=x.dtype, device=x.device)
        sv, sw, sr, sq = (self.sigma * c for c in self.SCALE)
        x[:, 0:3] += sv * n[:, 0:3]
        x[:, 3:6] += sw * n[:, 3:6]
        x[:, 6:9] += sr * n[:, 6:9]
        q = x[:, 9:13] + sq * n[:, 9:13]
        x[:, 9:13] = q / q.norm(dim=1, keepdim=True)


class FleetLoop:
    """Closed-loop state of one rank's shard and its per-step sequence."""

    def __init__(self, stepper, x0: torch.Tensor, N: int, dt: float, ekf: bool = False, ekf_substeps: int = 5,
                 covariances: Optional[tuple] = None, publisher=None, noise: Optional[MeasurementNoise] = None):
        B = x0.shape[0]
        dev = x0.device
        f64 = dict(dtype=torch.float64, device=dev)
        self.stepper, self.N, self.dt, self.pub, self.noise = stepper, N, dt, publisher, noise
        self.x0 = x0.clone()
        self.u0 = torch.zeros((B, 4), **f64)
        self.traj = torch.zeros((B, N + 1, 15), **f64)
        self.diag = torch.zeros((B, 6), **f64)
        self.status = torch.zeros((B,), dtype=torch.int32, device=dev)
        self.ekf = ekf
        self.ekf_substeps = ekf_substeps
        if ekf:
            if covariances is None:
                raise ValueError("the EKF needs (W, V, P0)")
            W, V, P0 = (np.asarray(a, dtype=np.float64) for a in covariances)
            self.W = torch.from_numpy(W.copy()).to(dev)
            self.V = torch.from_numpy(V.copy()).to(dev)
            self.P = torch.from_numpy(np.repeat(P0[None], B, axis=0)).to(dev)
            self.xe = self.x0[:, :13].clone()
            self.u3 = torch.zeros((B, 3), **f64)
            self.z = self.x0[:, 6:13].clone()
        self.gathered = None

    def step(self):
        if self.ekf:
            # propagate under the control applied last (u(t0) of the previous
            # plan), update with the measurement on the last substep
            self.u3.copy_(self.u0[:, :3])
            h = self.dt / self.ekf_substeps
            for j in range(self.ekf_substeps):
                self.stepper.ekf(h, self.xe, self.u3, self.P, self.z if j == self.ekf_substeps - 1 else None,
                                 self.W, self.V)
            self.x0[:, :13].copy_(self.xe)
        self.stepper.rti(self.x0, self.u0, self.traj, self.diag, self.status)
        if self.pub is not None:
            self.gathered = self.pub.publish(self.u0, self.diag)
        self.x0.copy_(self.traj[:, 1, :])
        if self.noise is not None:
            self.noise.apply(self.x0)
        if self.ekf:
            self.z.copy_(self.x0[:, 6:13])
