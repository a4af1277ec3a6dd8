"""Diagnostic: statuses / errors vs the oracle for each waves-per-agent setting on small
batches of several shapes (GPU).   python tools/quick_nw.py"""
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
import numpy as np  # noqa: E402
import oracle  # noqa: E402
import srbnmpc  # noqa: E402
from srbnmpc import workload  # noqa: E402

if len(sys.argv) > 1:                  # alternative build, e.g. libsrbnmpc_nodpp.so
    srbnmpc.LIB_PATH = os.path.join(os.path.dirname(srbnmpc.__file__), sys.argv[1])
    print("library", sys.argv[1])

k2 = json.load(open(os.path.join(ROOT, "tests", "golden", "kat2.json")))
for nw in (1, 2, 4):
    s = srbnmpc.BatchSolver(srbnmpc.default_params(4, 4), 1, 0)
    s.set_waves(nw)
    foot = np.repeat(np.asarray(k2["F"])[None], 4, 0)
    out = s.solve(np.asarray(k2["x0"])[None], np.asarray(k2["ref"])[None], foot[None], np.asarray(k2["obstacle"])[None])
    print(f"kat2 nw={s.waves()}: status {out['status'][0]} iters {out['iters'][0]} "
          f"qp err {np.abs(out['x_qp'][0, :24] - np.asarray(k2['logged_qp_x'])).max():.2e}", flush=True)
    s.close()
for (N, C, Ko, Kn, A) in [(4, 4, 1, 0, 8), (4, 2, 1, 0, 8), (10, 2, 3, 0, 16), (10, 2, 3, 8, 16), (20, 2, 3, 8, 16), (10, 4, 3, 0, 8)]:
    b = workload.make_batch(A, N, C, seed=5)
    r = oracle.solve_batch(oracle.params(N, C, K_obs=Ko, K_nbr=Kn), b["x0"], b["ref"], b["foot"], b["obstacles"],
                           b["nbr_state"], nthreads=8)
    for nw in (1, 2, 4):
        s = srbnmpc.BatchSolver(srbnmpc.default_params(N, C, K_obs=Ko, K_nbr=Kn), A, 0)
        s.set_waves(nw)
        try:
            out = s.solve(b["x0"], b["ref"], b["foot"], b["obstacles"], b["nbr_state"])
        except RuntimeError as e:
            print(f"N={N} C={C} K={Ko}+{Kn} nw={nw}: {e}"); continue
        e = np.abs(out["x"] - r["x"])[:, :6 * N].max()
        print(f"N={N} C={C} K={Ko}+{Kn} nw={s.waves()}: status ok {(out['status'] == r['status']).all()} "
              f"{np.bincount(out['status'].ravel(), minlength=5)} iters eq {(out['iters'] == r['iters']).mean():.2f} err {e:.2e}",
              flush=True)
        s.close()
