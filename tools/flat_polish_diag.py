"""Diagnostic (round 6): the fused polish's last acceptance test per agent, from a
-DSRB_DIAG_POLISH_OUT build (make lipvar TAG=<tag> LIPFLAGS='-DSRB_DIAG_POLISH_OUT [-DSRB_DIAG_FLAT_EQRES]'),
on test_knn_matches_bruteforce's K = 3 + 0 batch (the case round 5's generic-pointer build failed) and 3 + 8.
Prints the statuses against the oracle and, for the agents whose polish was rejected, which tests failed and
the equality residual the kernel computed.
    python tools/flat_polish_diag.py libsrbnmpc_<tag>.so [waves]"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
import srbnmpc  # noqa: E402

srbnmpc.use_library(sys.argv[1])
import oracle  # noqa: E402
from srbnmpc import workload  # noqa: E402

NAMES = ["primal", "active", "mult", "step", "eq", "eq_nonfinite", "ran"]
N, C, A = 10, 2, 512
for Ko, Kn in ((3, 0), (3, 8)):
    b = workload.make_batch(A, N, C, seed=3)
    p = srbnmpc.default_params(N, C, K_obs=Ko, K_nbr=Kn, use_nlp=1)
    s = srbnmpc.BatchSolver(p, A)
    if len(sys.argv) > 2:
        s.set_waves(int(sys.argv[2]))
    out = s.solve(b["x0"], b["ref"], b["foot"], b["obstacles"], b["nbr_state"])
    print(f"K {Ko}+{Kn}: waves {s.waves()}")
    s.close()
    op = oracle.params(N, C, K_obs=Ko, K_nbr=Kn)
    r = oracle.solve_batch(op, b["x0"], b["ref"], b["foot"], b["obstacles"], b["nbr_state"], nthreads=8)
    st = out["status"][:, 1]
    print(f"   GPU NLP statuses {np.bincount(st, minlength=5).tolist()}  oracle {np.bincount(r['status'][:, 1], minlength=5).tolist()}")
    bits = out["iters"][:, 0]
    eqr = out["obj"]
    ran = (bits & 64) != 0
    rej = ran & (st != 0)
    print(f"   polish ran on {ran.sum()} agents, rejected on {rej.sum()}")
    for i, nm in enumerate(NAMES[:6]):
        print(f"      test {nm:13s} failed on {int(((bits[rej] >> i) & 1 == 0).sum()) if i != 5 else int(((bits[rej] >> 5) & 1).sum())} of the rejected")
    if rej.any():
        e = eqr[rej]
        print(f"   rejected agents' equality residual: finite {np.isfinite(e).sum()}, min {np.nanmin(e):.3e}, "
              f"median {np.nanmedian(e):.3e}, max {np.nanmax(e):.3e}")
        print("   first rejected agents:", np.where(rej)[0][:10].tolist(), "bits", bits[rej][:10].tolist(),
              "eqr", [f"{v:.3e}" for v in e[:10]])
    acc = ran & (st == 0)
    if acc.any():
        print(f"   accepted agents' equality residual: max {eqr[acc].max():.3e}")
