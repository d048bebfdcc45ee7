"""The RCCL branch of bench.py on one GPU: launched exactly as the
driver launches N > 1 (torch.distributed.run, one rank per GPU, 127.0.0.1),
here with --nproc-per-node 1.  The rank joins an "nccl" (RCCL) process group,
publishes every step through all_gather_into_tensor, brackets the timed region
with barriers and takes the max over ranks by all_reduce -- the collectives of
the multi-GPU path, at world size 1.  Scaling is not measured here."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_rccl_branch_world1():
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "3", "--warmup", "1", "--batch", "512", "--no-cpu-baseline"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert out["config"]["backend"] == "nccl" and out["config"]["allgather"] is True
    assert out["n_gpus"] == 1 and out["value"] > 0
    assert out["status_nan"] == 0
