#!/usr/bin/env python3
"""bench.py -- NMPC RTI steps/s for the openKITE kite controller on MI355X.

Workload (BASELINE.json configs[2]): batch = 4096 independent kite NMPC
instances per GPU, N = 20 shooting intervals (tf = 1 s), M = 2 RK4 substeps,
full fp64 RTI (shift -> RK4 + forward sensitivities -> Gauss-Newton
condensing with fp64 MFMA -> interior-point QP -> expansion) per step.
Synthetic, seeded instances; closed loop: the next step's
measured state is the predicted state at t0 + dt of the current solution
(openkite_amd/fleet.py).

One process per GPU (torch.distributed / RCCL); the batch shards with no
data-path collective (weak scaling); after each step the per-instance
results (u0 + mpc_diagnostic) are all-gathered over RCCL, as a controller
fleet would publish them.  ``--gpus N`` without a launcher starts the N
ranks itself (torch.distributed.run as a child process, before this process
touches a GPU) and fails if the node has fewer than N GPUs.

Prints ONE JSON line on rank 0 (see the driver contract in the task).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP64_TFLOPS = 78.6        # MI355X fp64 vector = fp64 matrix (AMD spec)
PEAK_HBM_GBS = 8000.0
METRIC = "NMPC RTI steps/sec, batch=4096 N=20 horizon, 1/2/4/8 MI355X"


TIMING_STRIDE = 3


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 30 + 3 steps: the synthetic fleet is a transient from the launch state; in
    # the nominal loop kites start to fail from step ~45 on, in the oracle
    # exactly as on the GPU (profiles/r05j_oracle_long_loop.txt)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=4096, help="instances per GPU")
    ap.add_argument("--horizon", type=int, default=20)
    ap.add_argument("--substeps", type=int, default=2)
    ap.add_argument("--qp-iters", type=int, default=16)
    ap.add_argument("--qp-kernel", type=int, default=0,
                    help="0 auto (2 at N = 20, else 3), 1 condensed wave-scalar, 2 condensed MFMA-tiled, 3 multiple-shooting Riccati")
    ap.add_argument("--no-allgather", action="store_true")
    ap.add_argument("--fp32-sens", action="store_true",
                    help="RK4 + sensitivities in fp32, QP fp64 (BASELINE configs[3] mixed precision)")
    ap.add_argument("--ekf", action="store_true",
                    help="fuse the EKF estimate (kiteEKF.cpp) before every RTI step (BASELINE configs[4])")
    ap.add_argument("--wind-sweep", type=float, default=0.0, metavar="VMAX",
                    help="wind-field sweep: a seeded constant world-frame wind per instance, horizontal speed "
                         "up to VMAX m/s (kite_nmpc_set_wind; a build extension, the reference model has no "
                         "wind); 0 = no wind, the reference model.  The synthetic ~4.5 m/s kites stay in their "
                         "envelope over a long closed loop up to ~0.5 m/s (DESIGN 2.1)")
    ap.add_argument("--meas-noise", type=float, default=0.0, metavar="S",
                    help="disturbed plant: seeded Gaussian noise on every measured state (body velocity and rates "
                         "0.05 S, position 0.01 S, attitude ~0.01 S rad; openkite_amd/fleet.py MeasurementNoise), "
                         "so the controller's model no longer predicts the plant exactly; 0 = the nominal loop")
    ap.add_argument("--rate-bound", type=float, default=0.0, metavar="W",
                    help="binding state box: |omega_i| <= W rad/s on every node instead of the reference's 4 pi "
                         "(nmpf_node.cpp:59-63, never active on this workload); the condensed QP enforces it with "
                         "lazy rows, the multiple-shooting QP (--qp-kernel 3) with soft rows on every node; 0 = the "
                         "reference bounds")
    ap.add_argument("--qp-lm", type=float, default=None,
                    help="qp_kernel 3: Levenberg-Marquardt term (default: the config's 10); 0 with --soft-weight 1e6 "
                         "at N = 20 is the undamped every-node mode (DESIGN 2.1)")
    ap.add_argument("--soft-weight", type=float, default=None,
                    help="qp_kernel 3: exact-L1 weight of the state rows (default: the config's 1e3)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="budget of the CPU baseline sample")
    ap.add_argument("--latency-steps", type=int, default=1000,
                    help="warm single-kite steps of the single-thread CPU latency (BASELINE config 1)")
    return ap.parse_args(argv)


def synthetic_wind(B, offset, vmax):
    """Wind-field sweep: per global instance a seeded world-frame wind, horizontal
    speed U(0, vmax) in a uniform direction, vertical U(-0.2, 0.2) vmax (None for
    vmax = 0: no wind)."""
    if vmax <= 0.0:
        return None
    w = np.zeros((B, 3))
    for b in range(B):
        rng = np.random.default_rng(77_000_000 + offset + b)
        ang, sp = rng.uniform(0.0, 2 * math.pi), rng.uniform(0.0, vmax)
        w[b] = [sp * math.cos(ang), sp * math.sin(ang), rng.uniform(-0.2, 0.2) * vmax]
    return w


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


def gpu_single_kite_latency(args, ok, xs, steps=200, warm=20, episode=25):
    """One kite per context, the ROS node's use (nmpf_node.cpp:206-246 calls
    computeControl for its one kite): wall time of the host entry point
    kite_nmpc_step (state in, control + plan out, PCIe both ways, stream
    synchronised) over warm closed-loop steps.  Not `value` (which is batch
    throughput with inputs in HBM); reported beside the CPU oracle's
    single-thread batch-1 latency.

    The loop runs in episodes of one cold step (reset, not timed) and
    `episode` warm steps, episode e on kite xs[e % len(xs)] -- the CPU
    oracle's batch-1 latency is measured the same way (cpu_baseline).  An
    unbroken loop would not do: the synthetic plant (the plan's node 1) leaves
    the feasible region after ~45-150 steps and then feeds the controller a
    non-finite state, after which every step is a cold restart whose QP exits
    at once -- a different workload (loop length).  The first
    `warm` warm steps (graph capture, page-in) are not timed."""
    cfg = ok.default_config(N=args.horizon, M=args.substeps, qp_iters=args.qp_iters)
    cfg.qp_kernel = args.qp_kernel
    cfg.sens_fp32 = 1 if args.fp32_sens else 0
    apply_qp_options(cfg, args)
    g = ok.BatchNMPC(ok.load_properties(), cfg, 1)
    try:
        ts, nonfinite, e = [], 0, 0
        while len(ts) < warm + steps:
            g.reset()
            r = g.step(xs[e % xs.shape[0]][None].copy())   # the episode's cold step
            e += 1
            x = r["traj"][:, 1, :].copy()
            for i in range(episode):
                t0 = time.perf_counter()
                r = g.step(x)
                ts.append(time.perf_counter() - t0)
                x = r["traj"][:, 1, :].copy()
                if not np.isfinite(x).all():
                    nonfinite += 1
                    break
        t = np.array(ts[warm:warm + steps]) * 1e3
    finally:
        g.close()
    return {"median_ms": round(float(np.median(t)), 4), "p90_ms": round(float(np.percentile(t, 90)), 4),
            "steps": int(t.size), "episode": episode, "nonfinite_episodes": nonfinite,
            "api": "kite_nmpc_step (host arrays, synchronous), warm steps in episodes of "
                   f"{episode} after a reset"}


def apply_qp_options(cfg, args):
    """--rate-bound, --qp-lm, --soft-weight on a context config or on the
    oracle's node_config dict (which also takes the QP form of --qp-kernel)."""
    apply_rate_bound(cfg, args.rate_bound)
    if isinstance(cfg, dict):
        import openkite_amd as ok
        if ok.resolve_qp_kernel(args.qp_kernel, args.horizon) == 3:
            cfg["qp_form"] = 1
        if args.qp_lm is not None:
            cfg["lm"] = args.qp_lm
        if args.soft_weight is not None:
            cfg["soft_weight"] = args.soft_weight
    else:
        if args.qp_lm is not None:
            cfg.qp_lm = args.qp_lm
        if args.soft_weight is not None:
            cfg.qp_soft_weight = args.soft_weight
    return cfg


def apply_rate_bound(cfg, w):
    """--rate-bound: |omega_i| <= w on the states 3..5 of every node (a config
    object or the oracle's node_config dict); w <= 0 keeps the reference box."""
    if w <= 0.0:
        return cfg
    lb, ub = (cfg["lbx"], cfg["ubx"]) if isinstance(cfg, dict) else (cfg.lbx, cfg.ubx)
    for i in range(3, 6):
        lb[i], ub[i] = -w, w
    return cfg


def host_cpu_info():
    """What the CPU numbers ran on: the machine's CPUs, this process's CPU set
    and cgroup quota, and the thread count the box allots (OMP_NUM_THREADS)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except Exception:
        affinity = None
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()
            quota = None if q == "max" else round(int(q) / int(p), 2)
    except Exception:
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    return dict(model=model, nproc=os.cpu_count(), affinity_cpus=affinity, cgroup_cpu_quota=quota,
                omp_num_threads=int(omp) if omp and omp.isdigit() else None)


def cpu_baseline(args, x0_host, budget_s, wind=None):
    """The CPU oracle (oracle/kite_oracle.cpp, OpenMP over instances) on a
    bounded sample of the same workload: same instances, cold start + warm
    closed-loop steps, same N/M/K; plus the single-thread, batch-1 latency
    (BASELINE config 1).  The reference's own CasADi/IPOPT path cannot run
    here; these are the build's restatement of the RTI."""
    from oracle import ffi
    info = host_cpu_info()
    # the threads this job may use: the box allots OMP_NUM_THREADS CPUs to a
    # one-GPU job (nproc shows the whole machine); else this process's CPU set
    threads = info["omp_num_threads"] or info["affinity_cpus"] or os.cpu_count() or 1
    kp = ffi.load_params()
    cfgv = ffi.cfg_vector(apply_qp_options(ffi.node_config(N=args.horizon), args))
    N = args.horizon
    S = min(x0_host.shape[0], 64 * threads)
    x = x0_host[:S].copy()
    ws = None if wind is None else wind[:S]
    X = np.zeros((S, N + 1, 15)); U = np.zeros((S, N, 4))
    ffi.rti_step(kp, cfgv, N, args.substeps, args.qp_iters, x, X, U, warm=0, nthreads=threads, wind=ws)
    x = X[:, 1, :].copy()
    steps, t0 = 0, time.perf_counter()
    while True:
        ffi.rti_step(kp, cfgv, N, args.substeps, args.qp_iters, x, X, U, warm=1, nthreads=threads, wind=ws)
        x = X[:, 1, :].copy()
        steps += 1
        el = time.perf_counter() - t0
        if (el >= budget_s and steps >= 2) or steps >= 200:
            break
    # config 1: one kite, one thread, warm closed-loop steps; 40 kites x 25
    # steps (each kite restarted cold, its cold step not timed)
    lat, per_kite = [], 25
    kites = max(1, (args.latency_steps + per_kite - 1) // per_kite)
    X1 = np.zeros((1, N + 1, 15)); U1 = np.zeros((1, N, 4))
    for k in range(kites):
        x1 = x0_host[k % x0_host.shape[0]][None].copy()
        ffi.rti_step(kp, cfgv, N, args.substeps, args.qp_iters, x1, X1, U1, warm=0, nthreads=1)
        for _ in range(per_kite):
            x1 = X1[:, 1, :].copy()
            t = time.perf_counter()
            ffi.rti_step(kp, cfgv, N, args.substeps, args.qp_iters, x1, X1, U1, warm=1, nthreads=1)
            lat.append(time.perf_counter() - t)
    lat = np.array(lat[:args.latency_steps]) * 1e3
    return dict(value=S * steps / el, unit="RTI steps/s", cores=threads, kind="port",
                sample=f"{S} instances x {steps} warm closed-loop RTI steps (N={N}, M={args.substeps}, "
                       f"K<={args.qp_iters}), oracle/kite_oracle.cpp -O3 OpenMP {threads} threads, {el:.1f} s; "
                       "the reference's CasADi/IPOPT path cannot be built or run here (SURVEY.md 8(c))",
                host=info,
                latency_1thread_batch1=dict(median_ms=round(float(np.median(lat)), 4),
                                            p05_ms=round(float(np.percentile(lat, 5)), 4),
                                            p95_ms=round(float(np.percentile(lat, 95)), 4),
                                            steps=int(lat.size), rti_per_s=round(1e3 / float(np.median(lat)), 1),
                                            note=f"BASELINE configs[0] analogue: one kite, one thread, warm "
                                                 f"closed-loop steps ({kites} kites x {per_kite})"))


def run_config_tag(args):
    tag = dict(batch=args.batch, N=args.horizon, M=args.substeps, K=args.qp_iters,
               fp32_sens=bool(args.fp32_sens), ekf=bool(args.ekf), qp_kernel=args.qp_kernel)
    if args.wind_sweep > 0.0:
        tag["wind_sweep"] = args.wind_sweep
    if args.meas_noise > 0.0:
        tag["meas_noise"] = args.meas_noise
    if args.rate_bound > 0.0:
        tag["rate_bound"] = args.rate_bound
    if args.qp_lm is not None:
        tag["qp_lm"] = args.qp_lm
    if args.soft_weight is not None:
        tag["soft_weight"] = args.soft_weight
    return tag


def pmc_traffic(names, cfg_tag):
    """HBM bytes per launch of the kernel this run launches (one of `names`)
    from the newest committed PMC summary (profiles/<round>_pmc_hbm.json,
    tools/pmc_summary.py) whose recorded bench configuration is this run's;
    None if no profile matches."""
    import glob
    import re

    def session_key(f):
        # profiles/r05q_..., r05aa_...: round, then session letters (a..z, aa..)
        m = re.match(r"r(\d+)([a-z]*)", os.path.basename(f))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_hbm.json")), key=session_key)
    for f in reversed(files):
        d = json.load(open(f))
        if d.get("bench_config") != cfg_tag:
            continue
        ks = d.get("kernels", {})
        for name in sorted(ks):
            if name.split("<")[0] in names and "traffic_bytes" in ks[name]:
                return ks[name]["traffic_bytes"], os.path.relpath(f, ROOT) + f" ({name})"
    return None, "no PMC summary of this configuration"


def dominant_kernel_names(dom, qp_kernel):
    """rocprofv3 names of the kernel(s) behind the HIP-event phase `dom`."""
    if dom != "qp":
        return {"prologue": ("k_prologue",), "rk4_sens": ("k_rk4_sens2",),
                "condense": ("k_condense20", "k_condense")}.get(dom, (f"k_{dom}",))
    return {3: ("k_qp_ric",), 2: ("k_qp_tiled", "k_qp_lds"), 1: ("k_qp",)}[qp_kernel]


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def count_gpus(kfd_nodes=KFD_NODES, dev_dri="/dev/dri", env=None) -> int:
    """GPUs this process may use, counted WITHOUT any HIP call (no torch.cuda,
    no amdsmi fallback that initialises HIP): the KFD topology nodes with SIMDs
    (CPU nodes have none) whose render node /dev/dri/renderD<minor> exists and
    is accessible, capped by a *_VISIBLE_DEVICES list when one is set."""
    env = os.environ if env is None else env
    n = 0
    try:
        nodes = sorted(os.listdir(kfd_nodes))
    except OSError:
        nodes = []
    for d in nodes:
        props = {}
        try:
            with open(os.path.join(kfd_nodes, d, "properties")) as f:
                for line in f:
                    k, _, v = line.strip().partition(" ")
                    props[k] = v
        except OSError:
            continue
        try:
            if int(props.get("simd_count", "0")) <= 0:
                continue
            minor = int(props.get("drm_render_minor", "-1"))
        except ValueError:
            continue
        rn = os.path.join(dev_dri, f"renderD{minor}")
        if minor >= 0 and os.path.exists(rn) and os.access(rn, os.R_OK | os.W_OK):
            n += 1
    if not nodes:
        # no readable KFD topology: the accessible render nodes (one per GPU)
        try:
            n = sum(1 for e in os.listdir(dev_dri) if e.startswith("renderD")
                    and os.access(os.path.join(dev_dri, e), os.R_OK | os.W_OK))
        except OSError:
            n = 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None and v.strip() != "":
            n = min(n, len([t for t in v.split(",") if t.strip() != ""]))
    return n


def launch_ranks(args, count=count_gpus, call=subprocess.call) -> int:
    """--gpus N without a launcher: start N ranks (one per GPU) as a child
    torch.distributed.run, before this process touches any GPU (an exec or a
    fork after HIP initialisation is what this pool forbids)."""
    if "torch" in sys.modules:
        import torch
        assert not torch.cuda.is_initialized(), "bench.py: HIP initialised before the ranks were started"
    have = count()
    if have < args.gpus:
        print(f"bench.py: --gpus {args.gpus} requested but this node has {have} GPU(s)", file=sys.stderr)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return call(cmd, env=env)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
        sys.exit(2)

    import torch
    import torch.distributed as dist
    import openkite_amd as ok
    from openkite_amd import flops
    from openkite_amd.fleet import FleetLoop, GpuStepper, MeasurementNoise
    from openkite_amd.shard import Publisher, max_over_ranks, shard

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # under a launcher (torch.distributed.run sets WORLD_SIZE) the ranks always
    # join an RCCL group -- also at world 1, so the collective path (barrier,
    # publish all-gather, max over ranks) runs on a one-GPU box too
    distributed = "WORLD_SIZE" in os.environ
    if distributed:
        dist.init_process_group("nccl", device_id=dev)

    B, N = args.batch, args.horizon
    cfg = ok.default_config(N=N, M=args.substeps, qp_iters=args.qp_iters, device=local)
    cfg.qp_kernel = args.qp_kernel
    cfg.sens_fp32 = 1 if args.fp32_sens else 0
    apply_qp_options(cfg, args)
    ctx = ok.BatchNMPC(ok.load_properties(), cfg, B)
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)

    offset, count = shard(world * B, world, rank)      # weak scaling: B instances per GPU
    assert count == B
    x0_host = synthetic_x0(B, offset, ctx)
    wind = synthetic_wind(B, offset, args.wind_sweep)
    if wind is not None:
        ctx.set_wind(wind)
    pub = Publisher(B, dev, world) if distributed and not args.no_allgather else None
    noise = MeasurementNoise(args.meas_noise, dev, 91_000_000 + rank) if args.meas_noise > 0.0 else None
    loop = FleetLoop(GpuStepper(ctx), torch.from_numpy(x0_host).to(dev), N, cfg.dt, ekf=args.ekf,
                     covariances=ok.ekf_default_covariances() if args.ekf else None, publisher=pub, noise=noise)

    for _ in range(args.warmup):
        loop.step()
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    # kernel events on every TIMING_STRIDE-th timed step: a recorded step
    # carries six events between its kernels (~4.6 us each, measurement cost
    # inside the timed region); the sampled steps give the per-kernel means
    ctx.timing_start((args.steps + TIMING_STRIDE - 1) // TIMING_STRIDE, TIMING_STRIDE)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loop.step()
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    nrec, ksum = ctx.timing_read()
    kkt, iters = ctx.qp_stats()
    it_sum = ctx.qp_iteration_sum()
    b_steps, b_rows = ctx.state_bound_stats()
    status = loop.status.cpu().numpy()

    elapsed_max = max_over_ranks(elapsed, dev)
    total_rti = world * B * args.steps
    value = total_rti / elapsed_max

    if rank == 0:
        # mean over every instance of every timed step (device-side running
        # sums restarted by timing_start), not just the last step
        mean_it = it_sum / float(B * args.steps)
        ric = ok.resolve_qp_kernel(args.qp_kernel, N) == 3
        # k_qp_tiled (qp_kernel 2 at N = 20) skips most residual products (recursive
        # residuals): counted as a lower bound (flops.qp)
        rec = not ric and N == 20 and ok.resolve_qp_kernel(args.qp_kernel, N) == 2
        fl = flops.rti_ric(N, args.substeps, mean_it) if ric else flops.rti(N, args.substeps, mean_it, rec)
        kernels = ["prologue", "rk4_sens", "condense", "qp"]
        avg_ms = {k: ksum[k] / max(1, nrec) for k in kernels + ["qp_main"]}
        dom = max(kernels, key=lambda k: avg_ms[k])
        dom_flops = fl.get(dom, 0.0) * B
        # the QP phase also holds the expansion and the lazy-row launch: its
        # roofline kernel (k_qp_tiled / k_qp_lds / k_qp / k_qp_ric) is timed
        # alone by the context's sixth event (kite_nmpc_timing_read)
        dom_ms = avg_ms["qp_main"] if dom == "qp" else avg_ms[dom]
        achieved = dom_flops / (dom_ms * 1e-3) / 1e12 if dom_ms > 0 else 0.0
        alt = {}
        if dom == "qp" and not ric:
            qm = flops.qp_models(N, mean_it, rec)
            alt = {f"frac_{k}_count": round(qm[k] * B / (dom_ms * 1e-3) / 1e12 / PEAK_FP64_TFLOPS, 5)
                   for k in ("dense", "survey")}
        rti_flops = fl["total"] * B / (ksum["total"] / max(1, nrec) * 1e-3) / 1e12
        qk = ok.resolve_qp_kernel(args.qp_kernel, N)
        traffic, tsrc = pmc_traffic(dominant_kernel_names(dom, qk), run_config_tag(args))
        # the roof priced against is the fp64 compute peak (dense fp64 MFMA and
        # vector are both 78.6 TFLOP/s on gfx950 and share the fp64 datapath);
        # the SQ counters show the kernels bound by fp64 instruction issue and
        # dependency latency at one wave per SIMD, which is what `bound` says
        roofline = dict(bound="fp64 issue/latency (1 wave/SIMD)", achieved=round(achieved, 4),
                        peak=PEAK_FP64_TFLOPS, unit="TFLOP/s",
                        frac=round(achieved / PEAK_FP64_TFLOPS, 5), traffic=traffic,
                        kernel=dominant_kernel_names(dom, ok.resolve_qp_kernel(args.qp_kernel, N))[0],
                        launch_ms=round(dom_ms, 5), flops_per_launch=dom_flops, **alt,
                        note="fp64 compute roof (dense fp64 MFMA = vector peak on gfx950); the kernel is "
                             "latency-bound (dependent VALU/MFMA/LDS chains at 1 wave/SIMD); achieved = "
                             "flops_per_launch (openkite_amd/flops.py, causal count: structurally zero "
                             "blocks of the condensed C are not work) / launch_ms (HIP events around that "
                             "kernel alone on the step stream); frac_dense_count / frac_survey_count: the same "
                             "time priced with dense C and with SURVEY 8(d)'s F_qp; traffic = HBM bytes per "
                             f"launch from {tsrc}")
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args, x0_host, args.cpu_seconds, wind)
        # beside the CPU baseline only (the profiled runs pass --no-cpu-baseline and
        # must see the batch launches alone)
        lat1 = gpu_single_kite_latency(args, ok, x0_host[:40]) if world == 1 and not args.no_cpu_baseline else None
        workload = (f"batch={B}/GPU, N={N}, M={args.substeps}, full RTI fp64"
                    + (", fp32 sensitivities (BASELINE configs[3] precision)" if args.fp32_sens else "")
                    + (" + fused EKF (BASELINE configs[4])" if args.ekf else
                       " (BASELINE configs[2])" if N == 20 and not args.fp32_sens and wind is None and noise is None
                       and args.rate_bound <= 0.0 and args.qp_lm is None and args.soft_weight is None else "")
                    + (f", wind-field sweep |W_h| <= {args.wind_sweep} m/s per instance (build extension)"
                       if wind is not None else "")
                    + (f", disturbed plant: measurement noise S = {args.meas_noise}" if noise is not None else "")
                    + (f", binding state box |omega_i| <= {args.rate_bound} rad/s" if args.rate_bound > 0.0 else "")
                    + (f", multiple-shooting QP lm = {cfg.qp_lm:g}, soft weight {cfg.qp_soft_weight:g}"
                       if args.qp_lm is not None or args.soft_weight is not None else ""))
        out = {
            "metric": METRIC,
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
            "config": {"workload": workload, "ekf": bool(args.ekf),
                       "batch_per_gpu": B, "global_batch": world * B, "horizon_N": N, "rk4_substeps": args.substeps,
                       "qp_iter_cap": args.qp_iters, "parallelism": f"dp{world}",
                       "allgather": pub is not None, "wind_sweep_mps": args.wind_sweep,
                       "meas_noise": args.meas_noise, "rate_bound": args.rate_bound,
                       "qp_kernel": ok.resolve_qp_kernel(args.qp_kernel, N), "qp_lm": cfg.qp_lm,
                       "qp_soft_weight": cfg.qp_soft_weight,
                       # the measurement window: the synthetic loop is a transient
                       # (DESIGN 6), so numbers compare only at equal windows
                       "timed_steps": args.steps, "warmup_steps": args.warmup,
                       "timing_stride": TIMING_STRIDE,
                       "backend": dist.get_backend() if distributed else "none"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "gpu_latency_batch1": lat1,
            "kernel_ms_per_step": {k: round(v, 4) for k, v in avg_ms.items() if k != "qp_main"},
            "qp_main_kernel_ms_per_step": round(avg_ms["qp_main"], 4),
            "kernel_timing": {"recorded_steps": nrec, "stride": TIMING_STRIDE,
                              "note": "HIP events on every stride-th timed step (the kernel means above and "
                                      "roofline.launch_ms); the other steps run without events"},
            "interval_integrations_per_s": round(world * B * N / (avg_ms["rk4_sens"] * 1e-3), 1)
            if avg_ms["rk4_sens"] > 0 else None,
            "rti_tflops_all_kernels": round(rti_flops, 4),
            "qp_mean_iterations": round(mean_it, 3),
            "qp_converged_frac": round(float(np.mean(kkt < 1e-8)), 5),
            "status_nan": int(np.sum(status & 1)),
            "state_bounds": {"kite_steps_outside": b_steps, "rows_outside": b_rows,
                             "kite_steps": B * args.steps,
                             "note": "over the timed steps: committed plans leaving the state box |omega_i| <= "
                                     + (f"{args.rate_bound}" if args.rate_bound > 0.0 else "4 pi") + ", "
                                     "|q_i| <= 1.01 (nmpf_node.cpp:59-63; status bit 8) and their (node, state) pairs "
                                     "outside it" + ("; multiple-shooting QP: soft rows with xi > 0 at the accepted "
                                                     "solution" if ok.resolve_qp_kernel(args.qp_kernel, N) == 3
                                                     else "; condensed QP: after the lazy rows (DESIGN 4.4)")},
            "status_last_step": {name: int(np.sum((status & bit) != 0)) for name, bit in
                                 (("nan", 1), ("qp_not_converged", 2), ("state_bound", 8), ("rejected", 32),
                                  ("restart", 64))},
            "qp": "multiple-shooting QP, Riccati IPM (k_qp_ric)" if ric else "condensed QP (k_qp_tiled / k_qp_lds / k_qp)",
            "algorithmic_flops_per_launch": {("k_qp_ric" if ric else "qp"): fl["qp"] * B,
                                             "k_rk4_sens2": fl["rk4_sens"] * B},
            "run_config": run_config_tag(args),
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
