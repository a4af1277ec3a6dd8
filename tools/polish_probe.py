"""Polish acceptance probe on the GPU (tuning aid): solve a bench config's batch and print the NLP
status counts, iteration maxima, solve / polish kernel times.  SRB_POLISH_RHO (env) overrides the
polish regularisation for the run.   python tools/polish_probe.py <config> [qp_init]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "srb-cbf-nmpc_amd"))
import bench  # noqa: E402
import srbnmpc  # noqa: E402

cfg_id = int(sys.argv[1]); qp_init = int(sys.argv[2]) if len(sys.argv) > 2 else 1
cfg = bench.CONFIGS[cfg_id]
A, b, lo, hi = bench.rank_batch(cfg_id, cfg["agents"], 1, 0)
s = srbnmpc.BatchSolver(srbnmpc.default_params(cfg["N"], cfg["C"], K_obs=cfg["K_obs"], K_nbr=cfg["K_nbr"]), A)
s.set_qp_init(qp_init)
out = s.solve(b["x0"], b["ref"], b["foot"], b["obstacles"], b["nbr_state"])
times = []
for _ in range(3):
    out = s.solve(b["x0"], b["ref"], b["foot"], b["obstacles"], b["nbr_state"])
    times.append((s.last_kernel_ms()[1], s.last_polish_ms()))
st, it = out["status"], out["iters"]
print(f"config {cfg_id} rho={os.environ.get('SRB_POLISH_RHO', 'default')} qp_init={qp_init}: nlp status "
      f"{np.bincount(st[:, 1], minlength=5).tolist()} iters max {it.max(0).tolist()} mean {it.mean(0).round(2).tolist()} "
      f"solve/polish ms {np.median(times, 0).round(4).tolist()}  not-OPTIMAL agents {np.where(st[:, 1] != 0)[0][:12].tolist()}")
np.savez(os.path.join(ROOT, "gpurun_out", f"probe_c{cfg_id}_{os.environ.get('SRB_POLISH_RHO', 'd')}.npz"), **out)
