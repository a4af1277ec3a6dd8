"""Diagnostic (round 6): the agents of the corrupted-cost build (tools/stationarity_guard_check.py) that the
polish certificate still reports OPTIMAL more than 1e-4 from the oracle.  For each: the solver-independent KKT
certificate (tests/kkt.py) of the GPU point and of the oracle point against the TRUE problem, their objectives,
and the active obstacle rows -- a certified GPU point is a KKT point of the true problem (another local optimum
of the non-convex NLP, or the same one to the certificate's accuracy), which no stationarity test can reject.
    python tools/guard_slip_analysis.py gpurun_out/r06_guard_libsrbnmpc_corrupt.so.npz"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd"), os.path.join(ROOT, "tests")]
import oracle  # noqa: E402
from kkt import certify, nlp_rows  # noqa: E402
from srbnmpc import workload  # noqa: E402

d = np.load(sys.argv[1])
N, C, A, Ko, Kn = 10, 2, 512, 3, 8
b = workload.make_batch(A, N, C, seed=3)
p = oracle.params(N, C, K_obs=Ko, K_nbr=Kn)
xus = np.r_[0:6 * N, (6 + C) * N]
x, xo, st = d["x"], d["x_oracle"], d["status"]
e = np.abs(x[:, xus] - xo[:, xus]).max(1)
bad = np.where((st[:, 1] == 0) & (e > 1e-4))[0]
print(f"{len(bad)} OPTIMAL agents > 1e-4 from the oracle: {bad.tolist()}")
for a in bad:
    Pd, c, Aeq, beq, G, h = oracle.build_qp(p, b["x0"][a], b["ref"][a], b["foot"][a])
    obs, eps = oracle.select_obstacles(p, b["x0"][a], b["obstacles"], b["nbr_state"], int(a))
    gJ, hh = nlp_rows(N, C, Pd.size, G, h, obs, eps, p.vsat)
    out = []
    for name, xx in (("gpu", x[a]), ("oracle", xo[a])):
        cert = certify(Pd, c, Aeq, beq, gJ, hh, xx)
        g, _ = gJ(xx)
        act = np.where(np.abs(g - hh)[G.shape[0]:G.shape[0] + N * obs.shape[1]] < 1e-7)[0]
        f = 0.5 * Pd @ (xx * xx) + c @ xx
        out.append(f"{name}: stat_rel {cert['stat_rel']:.1e} prim {cert['prim']:.1e} eq {cert['eq']:.1e} "
                   f"obj {f:.9f} active obstacle rows {act.tolist()}")
    print(f"agent {a}: |dx| {e[a]:.2e}\n   " + "\n   ".join(out))
