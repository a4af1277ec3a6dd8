"""Diagnostic (round 6): where the selection kernel's time goes at configs[2] -- srb_select_device on the static
obstacle table alone (tables 1, grid), the neighbour snapshot alone (2, brute force) and both (3, the two waves of
one workgroup on the two tables), HIP-event timed on the launch stream, 200 launches each.
    python tools/knn_split_timing.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
import bench  # noqa: E402
import srbnmpc  # noqa: E402

dev = torch.device("cuda:0")
c = bench.CONFIGS[3]
A, b, _, _ = bench.rank_batch(3, c["agents"], 1, 0)
t = {k: torch.as_tensor(np.ascontiguousarray(v), dtype=torch.float64, device=dev) for k, v in b.items()}
s = srbnmpc.BatchSolver(srbnmpc.default_params(c["N"], c["C"], K_obs=c["K_obs"], K_nbr=c["K_nbr"]), A)
ko, kn = s.n_selected(t["obstacles"].shape[0], A)
sel = torch.zeros((A, ko + kn), dtype=torch.int32, device=dev)
st = torch.cuda.current_stream(dev)
for tables in (1, 2, 3, 1, 2, 3):
    for _ in range(20):
        s.select_device(t["x0"], t["obstacles"], t["nbr_state"], sel, tables=tables, stream=st.cuda_stream, obstacles_version=1)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(200)]
    for a, z in ev:
        a.record(st)
        s.select_device(t["x0"], t["obstacles"], t["nbr_state"], sel, tables=tables, stream=st.cuda_stream, obstacles_version=1)
        z.record(st)
    torch.cuda.synchronize()
    ms = np.array([a.elapsed_time(z) for a, z in ev])
    print(f"tables {tables}: median {np.median(ms) * 1e3:.1f} us, p10 {np.percentile(ms, 10) * 1e3:.1f} us")
s.close()
