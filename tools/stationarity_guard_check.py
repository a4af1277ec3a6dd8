"""Diagnostic (round 6): does the polish's stationarity test catch the defect class of the round-5 generic-pointer
build -- feasible, converged, dual-feasible polished points of the wrong objective reported OPTIMAL?
Builds (make lipvar): TAG=corrupt LIPFLAGS=-DSRB_DIAG_CORRUPT_COST (the fused polish's cost registers of the X
rows 1 % off, the test on) and TAG=corruptns LIPFLAGS='-DSRB_DIAG_CORRUPT_COST -DSRB_POLISH_STOL=1e300' (test
off).  Per library: NLP statuses and, on the agents reported OPTIMAL, the distance to the oracle's solution.
    python tools/stationarity_guard_check.py libsrbnmpc_<tag>.so"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
import srbnmpc  # noqa: E402

srbnmpc.use_library(sys.argv[1])
import oracle  # noqa: E402
from srbnmpc import workload  # noqa: E402

N, C, A, Ko, Kn = 10, 2, 512, 3, 8
b = workload.make_batch(A, N, C, seed=3)
s = srbnmpc.BatchSolver(srbnmpc.default_params(N, C, K_obs=Ko, K_nbr=Kn, use_nlp=1), A)
out = s.solve(b["x0"], b["ref"], b["foot"], b["obstacles"], b["nbr_state"])
s.close()
r = oracle.solve_batch(oracle.params(N, C, K_obs=Ko, K_nbr=Kn), b["x0"], b["ref"], b["foot"], b["obstacles"],
                       b["nbr_state"], nthreads=8)
xus = np.r_[0:6 * N, (6 + C) * N]
e = np.abs(out["x"][:, xus] - r["x"][:, xus]).max(1)
opt = out["status"][:, 1] == 0
np.savez(os.path.join(ROOT, "gpurun_out", f"r06_guard_{os.path.basename(sys.argv[1])}.npz"), x=out["x"], status=out["status"],
         x_oracle=r["x"], status_oracle=r["status"])
print(f"{sys.argv[1]}: GPU NLP statuses {np.bincount(out['status'][:, 1], minlength=5).tolist()}, oracle "
      f"{np.bincount(r['status'][:, 1], minlength=5).tolist()}")
print(f"   reported OPTIMAL: {int(opt.sum())}; of them > 1e-4 from the oracle: {int((e[opt] > 1e-4).sum())} "
      f"(max {e[opt].max() if opt.any() else 0:.2e})")
print(f"   not OPTIMAL: {int((~opt).sum())}; their (interior-point) results within {e[~opt].max() if (~opt).any() else 0:.2e} of the oracle")
