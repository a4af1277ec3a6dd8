"""Diagnostic (round 6): the round-4 whole-shape N = 20 build's OPTIMAL results that differ from the shipped
round-4 build's by more than 1e-4 (tools/r04_n20_compare.py) -- the solver-independent KKT certificate
(tests/kkt.py) of both points against the true problem, and their objectives.  A wrong point that certifies
would be another KKT point of the non-convex NLP; one that does not is what the round-6 polish certificate rejects.
    python tools/r04_n20_certify.py gpurun_out/r06_r04n20_base.npz gpurun_out/r06_r04n20_whole.npz"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd"), os.path.join(ROOT, "tests")]
import oracle  # noqa: E402
from kkt import certify, nlp_rows  # noqa: E402
from srbnmpc import workload  # noqa: E402

a, w = np.load(sys.argv[1]), np.load(sys.argv[2])
N, C, A, Ko, Kn = 20, 2, 2048, 3, 8
b = workload.make_batch(A, N, C, seed=0)          # the round-4 workload generates the same batch
p = oracle.params(N, C, K_obs=Ko, K_nbr=Kn)
xus = np.r_[0:6 * N, (6 + C) * N]
sa, sw = a["on_status"][:, 1], w["on_status"][:, 1]
e = np.abs(a["on_x"][:, xus] - w["on_x"][:, xus]).max(1)
bad = np.where((sa == 0) & (sw == 0) & (e > 1e-4))[0]
rows = []
for i in bad:
    Pd, c, Aeq, beq, G, h = oracle.build_qp(p, b["x0"][i], b["ref"][i], b["foot"][i])
    obs, eps = oracle.select_obstacles(p, b["x0"][i], b["obstacles"], b["nbr_state"], int(i))
    gJ, hh = nlp_rows(N, C, Pd.size, G, h, obs, eps, p.vsat)
    r = []
    for xx in (a["on_x"][i], w["on_x"][i]):
        cert = certify(Pd, c, Aeq, beq, gJ, hh, xx)
        r += [cert["stat_rel"], cert["prim"], 0.5 * Pd @ (xx * xx) + c @ xx]
    rows.append(r)
rows = np.array(rows)
print(f"{len(bad)} agents OPTIMAL in both builds and > 1e-4 apart (max {e[bad].max():.2e})")
print(f"  shipped build : stat_rel max {rows[:, 0].max():.1e}, prim max {rows[:, 1].max():.1e}")
print(f"  whole shape   : stat_rel min {rows[:, 3].min():.1e} median {np.median(rows[:, 3]):.1e} max {rows[:, 3].max():.1e}, "
      f"prim max {rows[:, 4].max():.1e}")
print(f"  objective whole - shipped: min {(rows[:, 5] - rows[:, 2]).min():.2e}, median {np.median(rows[:, 5] - rows[:, 2]):.2e}")
print(f"  whole-shape points that certify (stat_rel < 1e-6): {int((rows[:, 3] < 1e-6).sum())}")
