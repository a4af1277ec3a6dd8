"""Round 6: term rows and reduced matrix stored in fp32 (fp64 accumulation, the fp64
refinement against the stored matrix) -- measured by the diagnostic build that rounds every stored entry to fp32
(make lipvar TAG=r32 LIPFLAGS=-DSRB_DIAG_ROUND32).  Config 5 (configs[4]'s shape) and configs[2]: NLP statuses
against the oracle, iterations, |x - oracle| in X, U, s, kernel time.
    python tools/round32_check.py libsrbnmpc_r32.so"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
import srbnmpc  # noqa: E402

srbnmpc.use_library(sys.argv[1])
import bench  # noqa: E402
import oracle  # noqa: E402

for cfg in (5, 3):
    c = bench.CONFIGS[cfg]
    N, C = c["N"], c["C"]
    A, b, _, _ = bench.rank_batch(cfg, c["agents"], 1, 0)
    args = (b["x0"], b["ref"], b["foot"], b["obstacles"], b["nbr_state"])
    xus = np.r_[0:6 * N, (6 + C) * N]
    r = oracle.solve_batch(oracle.params(N, C, K_obs=c["K_obs"], K_nbr=c["K_nbr"]), *args, nthreads=16)
    s = srbnmpc.BatchSolver(srbnmpc.default_params(N, C, K_obs=c["K_obs"], K_nbr=c["K_nbr"], use_nlp=1), A)
    out = s.solve(*args)
    ks = []
    for _ in range(10):
        s.solve(*args)
        ks.append(s.last_kernel_ms()[1])
    s.close()
    st = out["status"]
    e = np.abs(out["x"][:, xus] - r["x"][:, xus]).max(1)
    print(f"{sys.argv[1]} config {cfg}: kernel {np.median(ks):.4f} ms; NLP statuses {np.bincount(st[:, 1], minlength=5).tolist()} "
          f"(oracle {np.bincount(r['status'][:, 1], minlength=5).tolist()}); statuses == oracle {int((st == r['status']).all(1).sum())}/{A}; "
          f"iters mean {out['iters'].mean(0).round(2).tolist()} max {out['iters'].max(0).tolist()} (oracle mean "
          f"{r['iters'].mean(0).round(2).tolist()}); |x - oracle| max {e.max():.2e}, agents > 1e-4: {int((e > 1e-4).sum())}", flush=True)
