"""Diagnostic (round 6): the SRB-12 Riccati accuracy floor.  At tol_final 1e-9 (round 4's value;
the product uses 1e-8) the GPU's interior point ran into MAXIT on a few stand agents where the oracle's dense LU
converged.  Per library and tol_final: statuses, NLP iterations and the forces against the oracle's tight run, on
1024 stand agents (seed 21, the failing batch) and 1024 trot agents.
    python tools/srb12_tolfinal.py libsrbnmpc_<tag>.so"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
import srbnmpc  # noqa: E402

srbnmpc.use_library(sys.argv[1])
import oracle  # noqa: E402
from srbnmpc import srb12, workload  # noqa: E402

N, A = 10, 1024
for gait in ("stand", "trot"):
    b = workload.make_batch12(A, N, gait, seed=21)
    pt = oracle.params12(N, K_obs=3, K_nbr=8, tol=1e-9, tol_final=1e-11, qp_maxit=80, nlp_maxit=80, polish=0)
    t = oracle.solve_batch12(pt, b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
    tok = (t["status"] == 0).all(1) | ((t["status"][:, 0] == 4) & (t["status"][:, 1] == 0))
    for tf, pol in ((1e-8, 1), (1e-9, 1), (1e-9, 0), (1e-10, 0)):
        p = srb12.default_params(N, K_obs=3, K_nbr=8)
        p.tol_final = tf
        p.polish = pol
        s = srb12.Solver12(p, A)
        out = s.solve(b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
        s.close()
        st = out["status"][:, 1]
        e = np.abs(out["x"][:, 12 * N:24 * N] - t["x"][:, 12 * N:24 * N]).max(1)
        ok = (st == 0) & tok
        print(f"{sys.argv[1]} {gait} tol_final {tf:g} polish {pol}: NLP statuses {np.bincount(st, minlength=5).tolist()}, "
              f"iters mean {out['iters'][:, 1].mean():.2f} max {out['iters'][:, 1].max()}; forces vs tight run (both "
              f"converged, {int(ok.sum())}) max {e[ok].max():.2e} N", flush=True)
