"""Multi-controller (multi-GPU) plumbing: one controller shard per GPU, one process per GPU.

The reference runs `clusterSize` controllers side by side; each keeps its own ShardingContainerPoolBalancerState
whose slots hold `1/clusterSize` of every invoker's memory (SCPB:485-507, updateCluster SCPB:561-584) and schedules
only the activations it receives.  The shards never exchange scheduling state, so the data path has no collective
(weak scaling).  What the controllers do share is invoker health: every controller consumes the same health topic
(InvokerPool, SCPB:355-358).  Here that is one all-gather of the health vector between batches (configs[4]: "health
all-gathered every batch"); a shard adopts rank 0's view, which equals its own when the views agree (they do unless a
health ping is in flight), and applies it through owgs_update_health_device (updateInvokers, SCPB:512-551) before the
batch's releases and publishes.  `health_schedule` gives every batch its own vector (a changing set of unresponsive
invokers), the same on every shard.

Works with any torch.distributed backend: RCCL ("nccl") on the GPUs, gloo on the CPU (tests/test_distributed.py).
"""
from __future__ import annotations

import os

import numpy as np


def env_rank() -> tuple[int, int, int]:
    """(rank, world, local_rank) from the torch.distributed.run environment (defaults: single process)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_workload(name: str, rank: int, world: int, n_activations: int | None = None, **kw):
    """The workload of controller shard `rank` of `world` (shared cluster, own stream, clusterSize = world)."""
    from . import workload as W

    return W.config(name, n_activations=n_activations, shard=rank, n_shards=world, **kw)


class HealthExchange:
    """All-gathers the invoker health vector (uint8 InvokerState codes) across controller shards."""

    def __init__(self, dist, health, world: int, collective: bool | None = None):
        """`collective`: issue the all-gather through `dist` (default: when world > 1).  At world 1 with a real
        process group (bench.py --rccl) it runs RCCL's all-gather on one rank, so the N = 1 lease exercises the same
        collective, streams and ordering as the multi-GPU cadence."""
        import torch

        self.dist, self.health, self.world = dist, health, world
        self.collective = (world > 1) if collective is None else bool(collective)
        if self.collective and dist is None:
            raise ValueError("a collective health exchange needs a process group")
        self.flat = torch.empty(world * health.numel(), dtype=health.dtype, device=health.device)
        self.gathered = self.flat.view(world, health.numel())

    def exchange(self, view=None):
        """All-gathers this shard's health view (default: the initial vector) and returns the agreed one (rank 0's
        row) as a tensor on the health device."""
        v = self.health if view is None else view
        if self.collective:
            self.dist.all_gather_into_tensor(self.flat, v)
        else:
            self.gathered[0].copy_(v)
        return self.gathered[0]

    def exchange_into(self, view, flat):
        """As exchange, into a caller's buffer of world * n bytes (one per batch: exchanges of later batches can run
        ahead on another stream while earlier batches still read theirs); returns the agreed row (rank 0's)."""
        if self.collective:
            self.dist.all_gather_into_tensor(flat, view)
        else:
            flat[:view.numel()].copy_(view)
        self.gathered.copy_(flat.view(self.world, -1))  # (diagnostics: disagreeing_ranks reads the last exchange)
        return flat[:view.numel()]

    def disagreeing_ranks(self) -> list[int]:
        """Ranks whose last gathered view differs from rank 0's (diagnostics)."""
        g = self.gathered.cpu().numpy()
        return [r for r in range(self.world) if not np.array_equal(g[r], g[0])]


def max_over_ranks(dist, values, device) -> list[float]:
    """Element-wise max of a list of floats over all ranks (step time, error flags, kernel time)."""
    import torch

    v = torch.tensor([float(x) for x in values], dtype=torch.float64, device=device)
    if dist is not None:
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
    return [float(x) for x in v.cpu()]


def whole_job_rate(n_per_shard: int, world: int, t_step_max: float) -> float:
    """Weak-scaling throughput: all shards' decisions divided by the slowest shard's step time."""
    return world * n_per_shard / t_step_max


def health_schedule(inv_status, n_batches: int, churn: float = 0.01, seed: int = 0xC4A17) -> np.ndarray:
    """Invoker health per batch [n_batches, n_invokers] (InvokerState codes): the cluster's vector with, in every batch
    after the first, a different `churn` fraction of the invokers Unresponsive (pings lost, InvokerSupervision.scala:
    339-365) -- the same on every controller shard, as the health topic is."""
    from .balancer import UNRESPONSIVE

    base = np.asarray(inv_status, dtype=np.uint8)
    out = np.repeat(base[None, :], max(n_batches, 1), axis=0)
    n = len(base)
    for b in range(1, n_batches):
        rng = np.random.Generator(np.random.PCG64([seed, b]))
        out[b, rng.choice(n, size=max(1, int(churn * n)), replace=False)] = UNRESPONSIVE
    return out
