"""Diagnostic (round 6): run the LDS-bounds build (make fullvar TAG=ldsck
VARFLAGS=-DSRB_DIAG_LDS_CHECK) over every instance family the product launches -- one, two and four waves per
agent, stored and folded obstacle rows, compiled and run-time shapes, the fused polish and the polish kernel --
and count the agents whose checks failed (QP status 1000 + flag bits, srb_kernels.hip LCK).
    python tools/lds_check_scan.py [libsrbnmpc_ldsck.so]"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
import srbnmpc  # noqa: E402

srbnmpc.use_library(sys.argv[1] if len(sys.argv) > 1 else "libsrbnmpc_ldsck.so")
from srbnmpc import workload  # noqa: E402

CASES = [  # N, C, K_obs, K_nbr, agents, waves (0 automatic), polish_fused
    (10, 2, 3, 8, 1024, 0, 1), (10, 2, 3, 0, 64, 0, 1), (20, 2, 3, 8, 2048, 0, 1), (10, 2, 3, 8, 96, 4, 1),
    (10, 2, 3, 8, 512, 2, 1), (4, 4, 1, 0, 16, 0, 1), (4, 2, 1, 0, 16, 1, 1), (10, 4, 3, 0, 64, 1, 1),
    (20, 2, 3, 0, 24, 0, 1), (10, 2, 0, 0, 32, 0, 1), (10, 2, 16, 16, 256, 1, 1), (16, 2, 3, 8, 128, 1, 1),
    (10, 2, 3, 8, 512, 1, 0), (20, 2, 3, 8, 256, 2, 0), (24, 2, 3, 0, 64, 0, 1), (10, 2, 3, 8, 64, 0, 1),
]
bad_total = 0
for N, C, Ko, Kn, A, nw, pf in CASES:
    b = workload.make_batch(A, N, C, seed=N * 7 + Kn + A)
    s = srbnmpc.BatchSolver(srbnmpc.default_params(N, C, K_obs=Ko, K_nbr=Kn, use_nlp=1), A)
    s.set_waves(nw)
    s.set_option("polish_fused", pf)
    out = s.solve(b["x0"], b["ref"], b["foot"], b["obstacles"], b["nbr_state"])
    waves = s.waves()
    s.close()
    st = out["status"][:, 0]
    bad = st >= 1000
    bad_total += int(bad.sum())
    flags = sorted(set((st[bad] - 1000).tolist()))
    print(f"N {N:2d} C {C} K {Ko:2d}+{Kn:2d} A {A:5d} waves {waves} fused {pf}: flagged agents {int(bad.sum())}"
          + (f", flag bits {flags}" if flags else "") + f"; NLP statuses {np.bincount(out['status'][:, 1] % 1000, minlength=5).tolist()}")
print(f"total flagged agents: {bad_total}")
sys.exit(1 if bad_total else 0)
