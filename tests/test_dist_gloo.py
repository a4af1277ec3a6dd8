"""Multi-process (gloo, world_size 2, CPU) tests of the agent-sharded data path:
contiguous agent-major shards + one all-gather of the neighbour snapshot per cycle.
The GPU solve itself is exercised by the gpu tests; here each rank checks that what it
would hand the kernel (global neighbour table, its agent_offset, its shard of inputs)
reproduces the single-process batch exactly, and that the neighbour selection made from
the gathered table is the one the oracle makes for the whole batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n_total, q):
    import sys
    root = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "srb-cbf-nmpc_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from srbnmpc import dist as sdist, workload
        b = workload.make_batch(n_total, 10, 2, seed=42)
        lo, hi = sdist.shard_range(n_total, world, rank)
        local = torch.as_tensor(b["nbr_state"][lo:hi])
        ex = sdist.NeighbourExchange(n_total, world, rank, torch.device("cpu"))
        # the exchange object is reused every control cycle: a second cycle with moved agents
        # must return the new table from the same buffers
        moved = b["nbr_state"] + 0.5
        first = ex(torch.as_tensor(moved[lo:hi])).clone().numpy()
        gathered = ex(local).numpy().copy()
        ok_table = bool(np.array_equal(gathered, b["nbr_state"])) and bool(np.array_equal(first, moved))
        ok_table &= bool(np.array_equal(sdist.gather_states(local, n_total, world).numpy(), b["nbr_state"]))
        # neighbour choice of this shard from the gathered table == whole-batch choice
        p = oracle.params(10, 2, K_obs=2, K_nbr=4)
        ok_nbr = True
        for a in range(lo, hi, max(1, (hi - lo) // 5)):
            o1, _ = oracle.select_obstacles(p, b["x0"][a], b["obstacles"], gathered, a)
            o2, _ = oracle.select_obstacles(p, b["x0"][a], b["obstacles"], b["nbr_state"], a)
            ok_nbr &= bool(np.array_equal(o1, o2))
            ok_nbr &= bool(np.array_equal(oracle.select_idx(p, b["x0"][a], b["obstacles"], gathered, a),
                                          oracle.select_idx(p, b["x0"][a], b["obstacles"], b["nbr_state"], a)))
        # split selection around the collective (bench.py's multi-GPU step): the all-gather is
        # issued (start), the static obstacles are selected while it is in flight -- they need no neighbour
        # row --, then wait() and the neighbour selection; the two parts together == the one-pass selection
        p_st, p_nb = oracle.params(10, 2, K_obs=2, K_nbr=0), oracle.params(10, 2, K_obs=0, K_nbr=4)
        for cycle, tab in enumerate((moved, b["nbr_state"])):
            pend = ex.start(torch.as_tensor(tab[lo:hi]))
            st = [oracle.select_idx(p_st, b["x0"][a], b["obstacles"], None, a) for a in range(lo, hi)]
            got = pend.wait().numpy()
            ok_nbr &= bool(np.array_equal(got, tab))
            for i, a in enumerate(range(lo, hi)):
                nb = oracle.select_idx(p_nb, b["x0"][a], b["obstacles"], got, a)
                ok_nbr &= bool(np.array_equal(np.r_[st[i], nb], oracle.select_idx(p, b["x0"][a], b["obstacles"], tab, a)))
        # shard solve through the oracle with agent_offset == whole-batch rows
        r_local = oracle.solve_batch(p, b["x0"][lo:hi], b["ref"][lo:hi], b["foot"][lo:hi], b["obstacles"],
                                     gathered, agent_offset=lo)
        r_full = oracle.solve_batch(p, b["x0"], b["ref"], b["foot"], b["obstacles"], b["nbr_state"])
        ok_solve = bool(np.array_equal(r_local["x"], r_full["x"][lo:hi]))
        # max-over-ranks timing reduction used by bench.py
        t = torch.tensor([float(rank + 1)])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        q.put((rank, ok_table, ok_nbr, ok_solve, float(t.item()), hi - lo))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [9, 24])
def test_sharded_gather_world2(n_total):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    res.sort()
    assert sum(r[5] for r in res) == n_total
    for rank, ok_table, ok_nbr, ok_solve, tmax, _ in res:
        assert ok_table and ok_nbr and ok_solve, rank
        assert tmax == float(world)


def test_shard_ranges_cover():
    from srbnmpc.dist import shard_range
    for n in (1, 7, 8192):
        for w in (1, 2, 4, 8):
            spans = [shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1
