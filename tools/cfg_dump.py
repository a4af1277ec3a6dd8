"""Development check: solve one bench configuration's batch once on the GPU and save the
per-agent status / iterations / solution to gpurun_out/cfg<c>_gpu.npz, for comparison with the
oracle on the CPU (tools/cfg_compare.py).   python tools/cfg_dump.py [config]"""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
import numpy as np  # noqa: E402

import bench  # noqa: E402
import srbnmpc  # noqa: E402
from srbnmpc import workload  # noqa: E402

c = int(sys.argv[1]) if len(sys.argv) > 1 else 5
cfg = bench.CONFIGS[c]
A, N, C = cfg["agents"], cfg["N"], cfg["C"]
p = srbnmpc.default_params(N, C, K_obs=cfg["K_obs"], K_nbr=cfg["K_nbr"], use_nlp=1)
b = workload.make_batch(A, N, C, seed=1234)
s = srbnmpc.BatchSolver(p, A)
out = s.solve(b["x0"], b["ref"], b["foot"], b["obstacles"], b["nbr_state"] if cfg["K_nbr"] else None)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", f"cfg{c}_gpu.npz"), **{k: np.asarray(v) for k, v in out.items()})
st = np.asarray(out["status"])
print("config", c, "non-optimal agents", np.where((st != 0).any(1))[0].tolist(), flush=True)
