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


class NeighbourExchange:
    """The per-cycle all-gather of the [n_local, 4] neighbour-state rows of every rank into
    one [n_total, 4] table in global agent order, with every buffer allocated once: each
    rank's rows go into a padded [cmax, 4] slot of one flat receive buffer
    (all_gather_into_tensor: a single RCCL call, no per-step list or torch.cat).  With equal
    shards (n_total % world == 0) the receive buffer IS the table; otherwise the padding is
    squeezed out by one index_select into a preallocated table."""

    def __init__(self, n_total: int, world: int, rank: int, device, dtype=None, force_collective: bool = False):
        """force_collective: run the all-gather even with one rank (tests: the RCCL path on one GPU)."""
        import torch as _t
        dtype = dtype or _t.float64
        self.n_total, self.world, self.rank = n_total, world, rank
        self.force = bool(force_collective)
        self.counts = [shard_range(n_total, world, r)[1] - shard_range(n_total, world, r)[0] for r in range(world)]
        self.cmax = max(self.counts)
        self.send = _t.zeros((self.cmax, 4), dtype=dtype, device=device)
        self.recv = _t.zeros((world * self.cmax, 4), dtype=dtype, device=device)
        self.equal = all(c == self.cmax for c in self.counts)
        if not self.equal:
            rows = [r * self.cmax + i for r in range(world) for i in range(self.counts[r])]
            self.rows = _t.as_tensor(rows, dtype=_t.long, device=device)
            self.table = _t.zeros((n_total, 4), dtype=dtype, device=device)
        self.out = self.recv if self.equal else self.table     # the [n_total, 4] table wait() returns
        # gloo (CPU tests) has no all_gather_into_tensor on every torch build: list form there
        self.flat = dist.is_initialized() and dist.get_backend() != "gloo"

    def __call__(self, local_state: torch.Tensor) -> torch.Tensor:
        return self.start(local_state).wait()

    def start(self, local_state: torch.Tensor) -> "PendingExchange":
        """Issue the all-gather without waiting for it (async_op): the caller runs work that does not need
        the neighbour table -- the static-obstacle selection (bench.py) -- then .wait() on the handle.  With
        RCCL, wait() orders the caller's current stream after the collective without blocking the host, so
        the static selection kernel and the all-gather overlap on the GPU."""
        if self.world == 1 and not self.force:
            return PendingExchange(self, None, local_state)
        if local_state.shape[0] != self.counts[self.rank]:
            raise ValueError(f"rank {self.rank} holds {self.counts[self.rank]} agents, got {local_state.shape[0]} rows")
        self.send[:local_state.shape[0]].copy_(local_state)
        if self.flat:
            work = dist.all_gather_into_tensor(self.recv, self.send, async_op=True)
        else:
            work = dist.all_gather(list(self.recv.view(self.world, self.cmax, 4).unbind(0)), self.send, async_op=True)
        return PendingExchange(self, work, None)


class PendingExchange:
    """An all-gather in flight (NeighbourExchange.start); wait() returns the [n_total, 4] table."""

    def __init__(self, ex: NeighbourExchange, work, table):
        self.ex, self.work, self.table = ex, work, table

    def wait(self) -> torch.Tensor:
        if self.table is not None:
            return self.table
        self.work.wait()
        ex = self.ex
        if ex.equal:
            self.table = ex.recv
        else:
            torch.index_select(ex.recv, 0, ex.rows, out=ex.table)
            self.table = ex.table
        return self.table


def gather_states(local_state: torch.Tensor, n_total: int, world: int) -> torch.Tensor:
    """One-shot form of NeighbourExchange (allocates its buffers per call)."""
    if world == 1:
        return local_state
    return NeighbourExchange(n_total, world, dist.get_rank(), local_state.device, local_state.dtype)(local_state)
