"""Multi-GPU sharding of a QPPVM batch.

QPPVM instances are independent (one robot state, or one MPC rollout, per instance), so the
path partitions: one process per GPU, each rank solves a contiguous shard of the global
batch with no data-path collective (weak scaling). The only exchange is optional: an
all-gather of the per-rank torques so that every rank holds the whole batch's tau (e.g. a
central rollout selector). On GPUs that all-gather is RCCL over xGMI (backend "nccl"); on
CPU it is gloo, which is what the multi-process tests use.

Nothing here touches libwbq: the solve is whatever the caller runs on its shard.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class ShardPlan:
    """Balanced contiguous partition of ``total`` instances over ``world`` ranks; the first
    ``total % world`` ranks get one instance more (ragged shards are allowed)."""
    total: int
    world: int

    def __post_init__(self):
        if self.world < 1 or self.total < 0:
            raise ValueError(f"bad shard plan: total={self.total}, world={self.world}")

    def count(self, rank: int) -> int:
        base, rem = divmod(self.total, self.world)
        return base + (1 if rank < rem else 0)

    def start(self, rank: int) -> int:
        base, rem = divmod(self.total, self.world)
        return rank * base + min(rank, rem)

    def bounds(self, rank: int) -> tuple:
        s = self.start(rank)
        return s, s + self.count(rank)

    @property
    def max_count(self) -> int:
        return self.count(0)


def gather_shards(local, plan: ShardPlan, rank: int, group=None):
    """All-gather the per-rank row blocks ``local`` ([plan.count(rank), ...] torch tensor)
    into the global [plan.total, ...] tensor on every rank. Shards are padded to the
    largest one so that RCCL moves one contiguous buffer (all_gather_into_tensor)."""
    import torch
    import torch.distributed as dist

    if local.shape[0] != plan.count(rank):
        raise ValueError(f"rank {rank}: shard has {local.shape[0]} rows, plan says {plan.count(rank)}")
    mc = plan.max_count
    if local.shape[0] == mc:
        pad = local.contiguous()
    else:
        pad = torch.zeros((mc,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        pad[: local.shape[0]] = local
    if dist.get_backend(group) == "nccl":
        buf = torch.empty((plan.world * mc,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(buf, pad, group=group)
        parts = [buf[r * mc: r * mc + plan.count(r)] for r in range(plan.world)]
    else:
        bufs = [torch.empty_like(pad) for _ in range(plan.world)]
        dist.all_gather(bufs, pad, group=group)
        parts = [bufs[r][: plan.count(r)] for r in range(plan.world)]
    return torch.cat(parts, dim=0)


def max_over_ranks(values, device=None, group=None):
    """Element-wise max of a list of floats over all ranks (the bench's step timing)."""
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return [float(v) for v in t.cpu()]
