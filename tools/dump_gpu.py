"""Diagnostic: solve one bench configuration on the GPU and save the raw outputs (x_qp, x,
status, iters, sel) to an .npz, for offline comparison with the oracle on the CPU.

    python tools/dump_gpu.py <config> <out.npz> [agents]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "srb-cbf-nmpc_amd"))
import bench  # noqa: E402
import srbnmpc  # noqa: E402
from srbnmpc import workload  # noqa: E402

cfg = bench.CONFIGS[int(sys.argv[1])]
A = int(sys.argv[3]) if len(sys.argv) > 3 else cfg["agents"]
p = srbnmpc.default_params(cfg["N"], cfg["C"], K_obs=cfg["K_obs"], K_nbr=cfg["K_nbr"], use_nlp=1)
b = workload.make_batch(A, cfg["N"], cfg["C"], seed=1234)
s = srbnmpc.BatchSolver(p, A)
out = s.solve(b["x0"], b["ref"], b["foot"], b["obstacles"], b["nbr_state"])
np.savez_compressed(sys.argv[2], **out)
st = out["status"]
print(f"config {sys.argv[1]} A={A}: status counts QP {np.bincount(st[:, 0])}, NLP {np.bincount(st[:, 1])}, "
      f"iters max {out['iters'].max(0)}")
