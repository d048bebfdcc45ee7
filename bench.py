#!/usr/bin/env python3
"""bench.py -- NMPC RTI steps/s for the openKITE kite controller on MI355X.

Workload (BASELINE.json configs[2]): batch = 4096 independent kite NMPC
instances per GPU, N = 20 shooting intervals (tf = 1 s), M = 2 RK4 substeps,
full fp64 RTI (shift -> RK4 + forward sensitivities -> Gauss-Newton
condensing with fp64 MFMA -> interior-point QP -> expansion) per step.
Synthetic, seeded instances; closed loop: the next step's
measured state is the predicted state at t0 + dt of the current solution.

One process per GPU (torch.distributed / RCCL); the batch shards with no
data-path collective (weak scaling); after each step the per-instance
results (u0 + mpc_diagnostic) are all-gathered over RCCL, as a controller
fleet would publish them.

Prints ONE JSON line on rank 0 (see the driver contract in the task).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP64_TFLOPS = 78.6        # MI355X fp64 vector = fp64 matrix (AMD spec)
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=4096, help="instances per GPU")
    ap.add_argument("--horizon", type=int, default=20)
    ap.add_argument("--substeps", type=int, default=2)
    ap.add_argument("--qp-iters", type=int, default=16)
    ap.add_argument("--qp-kernel", type=int, default=0, help="0 auto, 1 wave-scalar, 2 MFMA-tiled")
    ap.add_argument("--no-allgather", action="store_true")
    ap.add_argument("--fp32-sens", action="store_true",
                    help="RK4 + sensitivities in fp32, QP fp64 (BASELINE configs[3] mixed precision)")
    ap.add_argument("--ekf", action="store_true",
                    help="fuse the EKF estimate (kiteEKF.cpp) before every RTI step (BASELINE configs[4])")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="budget of the CPU baseline sample")
    return ap.parse_args()


def synthetic_x0(B, offset, ctx):
    """Seeded per-instance perturbations of launch/simulator.launch:3; theta from
    findClosestPointOnPath on the GPU (kiteNMPF.cpp:358-391), thetadot = 0."""
    base = np.array([4.4, 0.44, 1.73, 0.81, -1.73, -1.53, -0.46, -2.68, 0.64, -0.0289, 0.1587, 0.4304, 0.8881])
    x = np.zeros((B, 15))
    for b in range(B):
        rng = np.random.default_rng(20261015 + offset + b)
        s = base.copy()
        s[0:3] += rng.uniform(-0.5, 0.5, 3)
        s[3:6] += rng.uniform(-0.3, 0.3, 3)
        s[6:9] += rng.uniform(-0.05, 0.05, 3)
        axis = rng.normal(size=3); axis /= np.linalg.norm(axis)
        ang = math.radians(5.0) * rng.uniform(0, 1)
        dq = np.array([math.cos(ang / 2), *(math.sin(ang / 2) * axis)])
        q = s[9:13]
        qn = np.array([q[0] * dq[0] - q[1:] @ dq[1:], *(np.cross(q[1:], dq[1:]) + q[0] * dq[1:] + dq[0] * q[1:])])
        s[9:13] = qn / np.linalg.norm(qn)
        x[b, :13] = s
    x[:, 13] = ctx.closest_point(x[:, 6:9])
    return x


def cpu_baseline(args, x0_host, budget_s):
    """The CPU oracle (oracle/kite_oracle.cpp, OpenMP over instances) on a
    bounded sample of the same workload: same instances, cold start + warm
    closed-loop steps, same N/M/K.  Returns the dict for the JSON line."""
    from oracle import ffi
    kp = ffi.load_params()
    cfgv = ffi.cfg_vector(ffi.node_config(N=args.horizon))
    try:
        threads = len(os.sched_getaffinity(0))
    except Exception:
        threads = os.cpu_count() or 1
    threads = max(1, min(threads, 16))
    S = min(x0_host.shape[0], 64 * threads)
    x = x0_host[:S].copy()
    N = args.horizon
    X = np.zeros((S, N + 1, 15)); U = np.zeros((S, N, 4))
    ffi.rti_step(kp, cfgv, N, args.substeps, args.qp_iters, x, X, U, warm=0, nthreads=threads)
    x = X[:, 1, :].copy()
    steps, t0 = 0, time.perf_counter()
    while True:
        ffi.rti_step(kp, cfgv, N, args.substeps, args.qp_iters, x, X, U, warm=1, nthreads=threads)
        x = X[:, 1, :].copy()
        steps += 1
        el = time.perf_counter() - t0
        if (el >= budget_s and steps >= 2) or steps >= 200:
            break
    return dict(value=S * steps / el, unit="RTI steps/s", cores=threads, kind="port",
                sample=f"{S} instances x {steps} warm closed-loop RTI steps (N={N}, M={args.substeps}, "
                       f"K<={args.qp_iters}), oracle/kite_oracle.cpp -O3 OpenMP {threads} threads, {el:.1f} s")


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/<round>_pmc_hbm.json, written by tools/pmc_summary.py from
    separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this bench)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_hbm.json")))
    for f in reversed(files):
        d = json.load(open(f)).get("kernels", {})
        for name in (f"k_{kernel}_tiled", f"k_{kernel}"):
            if name in d and "traffic_bytes" in d[name]:
                return d[name]["traffic_bytes"], os.path.relpath(f, ROOT) + f" ({name})"
    return None, "no PMC summary"


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import openkite_amd as ok
    from openkite_amd import flops
    from openkite_amd.shard import Publisher, max_over_ranks, shard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    B, N = args.batch, args.horizon
    cfg = ok.default_config(N=N, M=args.substeps, qp_iters=args.qp_iters, device=local)
    cfg.qp_kernel = args.qp_kernel
    cfg.sens_fp32 = 1 if args.fp32_sens else 0
    ctx = ok.BatchNMPC(ok.load_properties(), cfg, B)
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)

    offset, count = shard(world * B, world, rank)      # weak scaling: B instances per GPU
    assert count == B
    x0_host = synthetic_x0(B, offset, ctx)
    d_x0 = torch.from_numpy(x0_host).to(dev)
    d_u0 = torch.zeros((B, 4), dtype=torch.float64, device=dev)
    d_traj = torch.zeros((B, N + 1, 15), dtype=torch.float64, device=dev)
    d_diag = torch.zeros((B, 6), dtype=torch.float64, device=dev)
    d_status = torch.zeros((B,), dtype=torch.int32, device=dev)
    pub = Publisher(B, dev, world) if world > 1 and not args.no_allgather else None

    if args.ekf:
        W, V, P0 = ok.ekf_default_covariances()
        d_W = torch.from_numpy(W).to(dev); d_V = torch.from_numpy(V).to(dev)
        d_P = torch.from_numpy(np.repeat(P0[None], B, axis=0)).to(dev)
        d_xe = d_x0[:, :13].clone()
        d_u3 = torch.zeros((B, 3), dtype=torch.float64, device=dev)
        d_z = d_x0[:, 6:13].clone()

    def one_step():
        if args.ekf:
            # estimator (kiteEKF.cpp:75-126): propagate under the applied control,
            # update with the measured position + attitude of the plant (here the
            # model's own prediction), then the RTI from the estimate
            # (propagation in 5 steps of dt/5: one RK4 step of 0.05 s is too coarse
            # for the tether dynamics; the reference estimator runs at the
            # measurement rate)
            d_u3.copy_(d_u0[:, :3])
            for j in range(5):
                ctx.ekf_step_device(B, cfg.dt / 5, d_xe.data_ptr(), d_u3.data_ptr(), d_P.data_ptr(),
                                    d_z.data_ptr() if j == 4 else 0, d_W.data_ptr(), d_V.data_ptr())
            d_x0[:, :13].copy_(d_xe)
        ctx.step_device(d_x0.data_ptr(), d_u0.data_ptr(), d_traj.data_ptr(), 0, d_diag.data_ptr(),
                        d_status.data_ptr())
        if args.ekf:
            d_z.copy_(d_traj[:, 1, 6:13])
        if pub is not None:
            pub.publish(d_u0, d_diag)          # all ranks see every kite's u0 + diagnostics
        d_x0.copy_(d_traj[:, 1, :])        # closed loop: predicted state at t0 + dt

    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ctx.timing_start(args.steps)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    nrec, ksum = ctx.timing_read()
    kkt, iters = ctx.qp_stats()
    it_sum = ctx.qp_iteration_sum()
    status = d_status.cpu().numpy()

    elapsed_max = max_over_ranks(elapsed, dev)
    total_rti = world * B * args.steps
    value = total_rti / elapsed_max

    if rank == 0:
        # mean over every instance of every timed step (device-side running
        # sums restarted by timing_start), not just the last step
        mean_it = it_sum / float(B * args.steps)
        fl = flops.rti(N, args.substeps, mean_it)
        kernels = ["prologue", "rk4_sens", "condense", "qp"]
        avg_ms = {k: ksum[k] / max(1, nrec) for k in kernels}
        dom = max(kernels, key=lambda k: avg_ms[k])
        dom_flops = fl.get(dom, 0.0) * B
        achieved = dom_flops / (avg_ms[dom] * 1e-3) / 1e12 if avg_ms[dom] > 0 else 0.0
        rti_flops = fl["total"] * B / (ksum["total"] / max(1, nrec) * 1e-3) / 1e12
        traffic, tsrc = pmc_traffic(dom)
        roofline = dict(bound="mfma", achieved=round(achieved, 4), peak=PEAK_FP64_TFLOPS, unit="TFLOP/s",
                        frac=round(achieved / PEAK_FP64_TFLOPS, 5), traffic=traffic, kernel=dom,
                        note="fp64 compute roof (vector = matrix peak on gfx950); achieved = algorithmic flops "
                             "per launch (openkite_amd/flops.py) / mean launch time (HIP events on the step "
                             f"stream); traffic = HBM bytes per launch from {tsrc}")
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args, x0_host, args.cpu_seconds)
        out = {
            "metric": "NMPC RTI steps/sec, batch=4096 N=20 horizon, 1/2/4/8 MI355X",
            "value": round(value, 1),
            "unit": "RTI steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64" if not args.fp32_sens else "f64 (f32 sensitivities)",
            "data": "synthetic (seeded perturbations of launch/simulator.launch:3, umx_radian params)",
            "config": {"workload": (f"batch={B}/GPU, N={N}, M={args.substeps}, full RTI fp64"
                                    + (", fp32 sensitivities (BASELINE configs[3] precision)" if args.fp32_sens else "")
                                    + (" + fused EKF (BASELINE configs[4])" if args.ekf else
                                       " (BASELINE configs[2])" if N == 20 else "")),
                       "ekf": bool(args.ekf),
                       "batch_per_gpu": B, "global_batch": world * B, "horizon_N": N, "rk4_substeps": args.substeps,
                       "qp_iter_cap": args.qp_iters, "parallelism": f"dp{world}",
                       "allgather": bool(world > 1 and not args.no_allgather)},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "kernel_ms_per_step": {k: round(v, 4) for k, v in avg_ms.items()},
            "rti_tflops_all_kernels": round(rti_flops, 4),
            "qp_mean_iterations": round(mean_it, 3),
            "qp_converged_frac": round(float(np.mean(kkt < 1e-8)), 5),
            "status_nan": int(np.sum(status & 1)),
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
