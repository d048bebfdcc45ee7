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
