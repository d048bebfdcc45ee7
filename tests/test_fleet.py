"""The per-rank closed loop of bench.py (openkite_amd/fleet.py) sharded over
ranks on CPU: world_size 2 over gloo, the oracle as each rank's stepper.

shard -> [EKF] -> RTI step -> Publisher all-gather -> next measured state, for
3 closed-loop steps; the gathered u0 + diagnostics of every kite must equal,
bitwise and in rank order, the same loop run on the unsharded batch in one
process.  (On the GPU the stepper is GpuStepper on libkite_nmpc.so and the
all-gather runs over RCCL; the sequence is the same object.)
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from openkite_amd.fleet import FleetLoop
from openkite_amd.shard import Publisher, shard

N, M, K, DT = 8, 2, 16, 0.05
STEPS = 3


class OracleStepper:
    """The fleet-loop stepper interface on the CPU oracle (test only)."""

    def __init__(self, B):
        from oracle import ffi
        self.ffi = ffi
        self.kp = ffi.load_params()
        self.cfgv = ffi.cfg_vector(ffi.node_config(N=N))
        self.X = np.zeros((B, N + 1, 15))
        self.U = np.zeros((B, N, 4))
        self.warm = 0

    def rti(self, x0, u0, traj, diag, status):
        u, d, st = self.ffi.rti_step(self.kp, self.cfgv, N, M, K, x0.numpy().copy(), self.X, self.U, warm=self.warm,
                                     nthreads=1)
        self.warm = 1
        u0.copy_(torch.from_numpy(u)); diag.copy_(torch.from_numpy(d)); status.copy_(torch.from_numpy(st))
        traj.copy_(torch.from_numpy(self.X))

    def ekf(self, h, xe, u3, P, z, W, V):
        for b in range(xe.shape[0]):
            x, Pb = self.ffi.ekf_step(self.kp, xe[b].numpy(), u3[b].numpy(), h, P[b].numpy(),
                                      None if z is None else z[b].numpy(), W.numpy(), V.numpy())
            xe[b] = torch.from_numpy(x)
            P[b] = torch.from_numpy(Pb)


def initial_states(offset, count):
    from oracle import ffi
    cv = ffi.cfg_vector(ffi.node_config(N=N))
    xs = ffi.synthetic_states(count, offset=offset)
    x = np.zeros((count, 15)); x[:, :13] = xs
    for b in range(count):
        x[b, 13] = ffi.closest_point(cv, xs[b, 6:9])
    return torch.from_numpy(x)


def covariances():
    import openkite_amd as ok
    return ok.ekf_default_covariances()


def run_loop(offset, count, ekf, publisher=None):
    loop = FleetLoop(OracleStepper(count), initial_states(offset, count), N, DT, ekf=ekf,
                     covariances=covariances() if ekf else None, publisher=publisher)
    out = []
    for _ in range(STEPS):
        loop.step()
        out.append(loop.gathered.clone() if publisher is not None else torch.cat([loop.u0, loop.diag], dim=1))
    return out


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, B, ekf, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        off, cnt = shard(world * B, world, rank)
        out = run_loop(off, cnt, ekf, Publisher(cnt, "cpu", world))
        q.put((rank, [t.numpy() for t in out]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ekf", [False, True])
def test_sharded_fleet_equals_unsharded_world2_gloo(ekf):
    world, B = 2, 4
    want = run_loop(0, world * B, ekf)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, world, port, B, ekf, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in range(world):
        for step in range(STEPS):
            np.testing.assert_array_equal(res[rank][step], want[step].numpy(), err_msg=f"rank {rank} step {step}")
    assert np.all(np.isfinite(want[-1].numpy()[:, :4]))


def test_bench_refuses_more_gpus_than_present():
    """bench.py --gpus 2 on a node without 2 GPUs exits non-zero instead of
    measuring one GPU (the parent checks before touching a GPU)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if torch.cuda.device_count() >= 2:
        pytest.skip("node has >= 2 GPUs")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0
    assert "GPU" in r.stderr
    assert r.stdout.strip() == ""


def test_measurement_noise_disturbs_the_plant_reproducibly():
    """bench.py --meas-noise (fleet.MeasurementNoise): the measured state is the
    plan's node 1 plus seeded noise on the kite states only (theta / thetadot
    untouched, the attitude renormalised), the same draws for the same seed; with the
    oracle as the stepper the disturbed loop leaves the nominal one."""
    from openkite_amd.fleet import MeasurementNoise
    B = 4
    runs = []
    for noise_seed in (None, 5, 5, 6):
        x0 = initial_states(0, B)
        noise = None if noise_seed is None else MeasurementNoise(1.0, torch.device("cpu"), noise_seed)
        loop = FleetLoop(OracleStepper(B), x0, N, DT, noise=noise)
        xs = []
        for _ in range(2):
            loop.step()
            xs.append(loop.x0.clone())
            traj1 = loop.traj[:, 1, :]
            np.testing.assert_array_equal(loop.x0[:, 13:].numpy(), traj1[:, 13:].numpy())
            if noise is not None:
                np.testing.assert_allclose(loop.x0[:, 9:13].norm(dim=1).numpy(), 1.0, rtol=1e-14)
                d = (loop.x0[:, :13] - traj1[:, :13]).abs()
                assert d.max() > 0 and d.max() < 0.5
            else:
                np.testing.assert_array_equal(loop.x0.numpy(), traj1.numpy())
        runs.append(torch.stack(xs))
    assert torch.equal(runs[1], runs[2])                 # same seed, same draws
    assert not torch.equal(runs[1], runs[3])             # another seed
    assert not torch.equal(runs[0], runs[1])             # the noise reaches the loop
