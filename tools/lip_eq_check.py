"""Diagnostic (round 5): the LIP equality rows (X_k = Ad X_{k-1} + Bd U_k, u_k = F_k lambda_k, sum lambda = 1)
at the GPU's returned points, by status, next to the oracle's statuses (test_knn_matches_bruteforce's batch).
    python tools/lip_eq_check.py [--lib libsrbnmpc_<tag>.so]"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
import srbnmpc  # noqa: E402

if len(sys.argv) > 2 and sys.argv[1] == "--lib":
    srbnmpc.use_library(sys.argv[2])
import oracle  # noqa: E402
from srbnmpc import workload  # noqa: E402

N, C, A = 10, 2, 512
for Ko, Kn in ((3, 0), (3, 8)):
    b = workload.make_batch(A, N, C, seed=3)
    p = srbnmpc.default_params(N, C, K_obs=Ko, K_nbr=Kn, use_nlp=1)
    s = srbnmpc.BatchSolver(p, A)
    out = s.solve(b["x0"], b["ref"], b["foot"], b["obstacles"], b["nbr_state"])
    print("waves", s.waves())
    s.close()
    op = oracle.params(N, C, K_obs=Ko, K_nbr=Kn)
    r = oracle.solve_batch(op, b["x0"], b["ref"], b["foot"], b["obstacles"], b["nbr_state"], nthreads=8)
    Ad, Bd = oracle.lip(op)
    X = out["x"][:, :4 * N].reshape(A, N, 4); U = out["x"][:, 4 * N:6 * N].reshape(A, N, 2)
    L = out["x"][:, 6 * N:6 * N + C * N].reshape(A, N, C); F = b["foot"].reshape(A, N, 2, C)
    res = np.zeros(A)
    for a in range(A):
        prev = b["x0"][a]
        for k in range(N):
            res[a] = max(res[a], np.abs(X[a, k] - Ad @ prev - Bd @ U[a, k]).max(),
                         np.abs(U[a, k] - F[a, k] @ L[a, k]).max(), abs(L[a, k].sum() - 1))
            prev = X[a, k]
    print(f"K {Ko}+{Kn}: GPU statuses {np.bincount(out['status'][:, 1], minlength=5).tolist()}  oracle "
          f"{np.bincount(r['status'][:, 1], minlength=5).tolist()}")
    rej = np.where((out["status"][:, 1] == 4) & (r["status"][:, 1] == 0))[0]
    print("   GPU 4 / oracle 0 agents:", rej[:12].tolist())
    if Ko == 3 and Kn == 0:
        open(os.path.join(ROOT, "gpurun_out", "r05_rej_agents.txt"), "w").write(" ".join(map(str, rej[:3])))
    for st in (0, 4):
        m = out["status"][:, 1] == st
        if m.any():
            print(f"   GPU status {st}: equality residual max {res[m].max():.2e} median {np.median(res[m]):.2e}; "
                  f"|x - x_oracle| max {np.abs(out['x'][m] - r['x'][m]).max():.2e}")
