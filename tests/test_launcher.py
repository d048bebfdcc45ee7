"""bench.py's multi-GPU launcher on CPU: the GPU count comes from the KFD
topology with no HIP call, and launching the ranks never initialises HIP in
the parent (a fork/exec after HIP initialisation is what the pool forbids)."""
import os
import sys
import types

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _topology(tmp_path, nodes):
    kfd = tmp_path / "nodes"
    dri = tmp_path / "dri"
    dri.mkdir()
    for i, (simds, minor) in enumerate(nodes):
        d = kfd / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count {simds}\ndrm_render_minor {minor}\n")
        if minor >= 0:
            (dri / f"renderD{minor}").write_text("")
    return str(kfd), str(dri)


def test_count_gpus_from_kfd_topology(tmp_path):
    kfd, dri = _topology(tmp_path, [(0, -1), (1024, 128), (1024, 129), (1024, 130)])
    assert bench.count_gpus(kfd, dri, env={}) == 3
    os.remove(os.path.join(dri, "renderD130"))             # a GPU of the host not passed to this container
    assert bench.count_gpus(kfd, dri, env={}) == 2
    assert bench.count_gpus(kfd, dri, env={"HIP_VISIBLE_DEVICES": "0"}) == 1
    # no KFD topology: the accessible render nodes
    assert bench.count_gpus(str(tmp_path / "absent"), dri, env={}) == 2
    assert bench.count_gpus(str(tmp_path / "absent"), str(tmp_path / "nodri"), env={}) == 0


def test_launch_ranks_never_initialises_hip(tmp_path):
    import torch
    calls = []
    args = types.SimpleNamespace(gpus=2)
    rc = bench.launch_ranks(args, count=lambda: 2, call=lambda cmd, env: calls.append((cmd, env)) or 0)
    assert rc == 0 and len(calls) == 1
    cmd, env = calls[0]
    assert "torch.distributed.run" in cmd and "--nproc-per-node=2" in cmd and "127.0.0.1" in cmd
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert not torch.cuda.is_initialized()
    # too few GPUs: refused before anything is started
    calls.clear()
    assert bench.launch_ranks(types.SimpleNamespace(gpus=8), count=lambda: 1, call=lambda c, env: calls.append(c)) == 2
    assert not calls


def test_rate_bound_option_sets_the_box_on_both_sides():
    """--rate-bound W sets |omega_i| <= W in the context config and in the CPU
    baseline's oracle config alike, and is part of the run tag the PMC lookup
    matches on; 0 keeps the reference box."""
    import openkite_amd as ok
    from oracle import ffi
    args = bench.parse(["--rate-bound", "3", "--qp-kernel", "3"])
    cfg = bench.apply_rate_bound(ok.default_config(N=20), args.rate_bound)
    assert [cfg.lbx[i] for i in range(3, 6)] == [-3.0] * 3 and [cfg.ubx[i] for i in range(3, 6)] == [3.0] * 3
    d = bench.apply_rate_bound(ffi.node_config(N=20), args.rate_bound)
    assert list(d["lbx"][3:6]) == [-3.0] * 3 and list(d["ubx"][3:6]) == [3.0] * 3
    assert bench.run_config_tag(args)["rate_bound"] == 3.0
    ref = ok.default_config(N=20)
    assert bench.apply_rate_bound(ok.default_config(N=20), 0.0).ubx[3] == ref.ubx[3]
    assert "rate_bound" not in bench.run_config_tag(bench.parse([]))
    # the undamped every-node mode reaches both the context and the baseline
    a2 = bench.parse(["--qp-kernel", "3", "--qp-lm", "0", "--soft-weight", "1e6"])
    c2 = bench.apply_qp_options(ok.default_config(N=20), a2)
    assert c2.qp_lm == 0.0 and c2.qp_soft_weight == 1e6
    d2 = bench.apply_qp_options(ffi.node_config(N=20), a2)
    assert d2["qp_form"] == 1 and d2["lm"] == 0.0 and d2["soft_weight"] == 1e6
    assert bench.apply_qp_options(ffi.node_config(N=20), bench.parse([]))["qp_form"] == 0
    assert bench.run_config_tag(a2)["qp_lm"] == 0.0
