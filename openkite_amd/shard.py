"""Data-parallel sharding of the kite batch over GPUs.

NMPC instances are independent, so the batch is split into contiguous slices,
one process and one library context per GPU, with no collective on the data
path.  The only exchange is the optional per-step publish of the control
actions and diagnostics (u0 [B x 4] + mpc_diagnostic [B x 6], fp64) to every
rank -- what a central consumer of all kites would read -- as one all-gather
(RCCL over xGMI with the "nccl" backend; gloo on CPU for the tests).

Used by bench.py; tests/test_shard.py runs it with world_size 2 on gloo.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

PUB_COLS = 10      # u0 (4) | diagnostic (6: pos, vel, cost, theta, Uv, kkt-or-time)


def shard(global_batch: int, world: int, rank: int) -> tuple[int, int]:
    """(offset, count) of this rank's contiguous slice; slices differ by at most 1."""
    base, extra = divmod(global_batch, world)
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


class Publisher:
    """Per-step all-gather of [u0 | diag] rows of every rank, in rank order.

    Every rank must hold the same per-rank batch (the weak-scaling setup);
    the gathered tensor is (world * B, 10) with rank r's rows at r*B.
    """

    def __init__(self, batch_per_rank: int, device, world: int):
        self.world = world
        self.pub = torch.zeros((batch_per_rank, PUB_COLS), dtype=torch.float64, device=device)
        self.gathered = torch.zeros((world * batch_per_rank, PUB_COLS), dtype=torch.float64, device=device)
        self._views = list(self.gathered.chunk(world, dim=0))
        self._nccl = dist.is_initialized() and dist.get_backend() == "nccl"

    def publish(self, u0: torch.Tensor, diag: torch.Tensor) -> torch.Tensor:
        self.pub[:, :4].copy_(u0)
        self.pub[:, 4:].copy_(diag)
        if not dist.is_initialized():
            self.gathered.copy_(self.pub)
        elif self._nccl:
            dist.all_gather_into_tensor(self.gathered, self.pub)
        else:
            dist.all_gather(self._views, self.pub)
        return self.gathered


def max_over_ranks(seconds: float, device) -> float:
    """Wall time of the slowest rank (the job's time)."""
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
