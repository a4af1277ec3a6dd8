"""Multi-GPU sharding for the agent batch (one process per GPU, torch.distributed).

Agents are independent given the neighbour snapshot (src/A1_Sim.cpp:181 reads the
neighbour state once per MPC call, include/shared_structs.hpp:94), so the batch shards
agent-major in contiguous blocks.  The only exchange is the neighbour snapshot: each rank
all-gathers the [x, y, xdot, ydot] rows of every agent (32 B per agent; RCCL over xGMI
when the backend is "nccl", gloo in the CPU tests) before the solve; the kNN and the
inter-agent CBF rows then run locally on each GPU.  Ranks never exchange solutions.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n_total: int, world: int, rank: int):
    """Contiguous agent-major block of rank `rank` (sizes differ by at most one)."""
    lo = (n_total * rank) // world
    hi = (n_total * (rank + 1)) // world
    return lo, hi


def gather_states(local_state: torch.Tensor, n_total: int, world: int) -> torch.Tensor:
    """All-gather the [n_local, 4] neighbour-state rows of every rank -> [n_total, 4]
    (rank order == global agent order).  One collective per control cycle."""
    if world == 1:
        return local_state
    counts = [shard_range(n_total, world, r)[1] - shard_range(n_total, world, r)[0] for r in range(world)]
    cmax = max(counts)
    buf = torch.zeros((cmax, 4), dtype=local_state.dtype, device=local_state.device)
    buf[:local_state.shape[0]] = local_state
    out = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(out, buf)
    return torch.cat([o[:c] for o, c in zip(out, counts)], 0)
