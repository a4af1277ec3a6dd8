"""Diagnostic (round 6): the fused polish's reduced stationarity ratio max|Z'(grad f + J_A' z_A)| / max(1, |grad f|)
at every accepted polish, from a build with -DSRB_DIAG_POLISH_OUT -DSRB_POLISH_STOL=1e300 (make lipvar TAG=stdiag):
obj carries the ratio, iters[:, 0] the acceptance bits (srb_kernels.hip SRB_POLISH_DIAG).  Bench configs 3 and 5.
    python tools/stationarity_scan.py libsrbnmpc_stdiag.so"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
import srbnmpc  # noqa: E402

srbnmpc.use_library(sys.argv[1])
import bench  # noqa: E402

for cfg in (3, 5):
    c = bench.CONFIGS[cfg]
    A, b, _, _ = bench.rank_batch(cfg, c["agents"], 1, 0)
    s = srbnmpc.BatchSolver(srbnmpc.default_params(c["N"], c["C"], K_obs=c["K_obs"], K_nbr=c["K_nbr"], use_nlp=1), A)
    out = s.solve(b["x0"], b["ref"], b["foot"], b["obstacles"], b["nbr_state"])
    s.close()
    st, bits, ratio = out["status"][:, 1], out["iters"][:, 0], out["obj"]
    acc = (st == 0) & ((bits & 64) != 0)
    q = np.sort(ratio[acc])[::-1]
    print(f"config {cfg}: {int(acc.sum())} accepted polishes; stationarity ratio max {q[0]:.2e}, "
          f"10 largest {[float(f'{v:.2e}') for v in q[:10]]}, median {np.median(q):.2e}; "
          f"above 1e-7: {int((q > 1e-7).sum())}, above 1e-8: {int((q > 1e-8).sum())}")
    top = np.where(acc)[0][np.argsort(-ratio[acc])[:5]]
    print("   agents", top.tolist(), "iters", out["iters"][top, 1].tolist())
